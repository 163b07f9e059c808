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

#include "fft_pk.h"
#include "gsdr_internal.h"
#include "gsdr_stream_internal.h"

// The reference loop is compiled for x86-64 without FMA contraction; keep every
// a*b+c of the restatement as two roundings.
#pragma clang fp contract(off)

namespace
{

#ifndef GSDR_TRK_THREADS
#define GSDR_TRK_THREADS 512
#endif
constexpr int kTrkThreads = GSDR_TRK_THREADS;
constexpr int kMaxCn0 = 64;         // cn0_samples capacity
constexpr int kMaxTrkTaps = 5;
constexpr int kMaxCodeFloats = 16384;
constexpr int kPreambleLen = 160;   // GPS_CA_PREAMBLE_LENGTH_SYMBOLS (GPS_L1_CA.h:61)
constexpr int kMaxSmoother = 32;             // Dll_Pll_Conf::smoother_length cap (high_dyn histories)
#ifndef GSDR_TRK_SPL
#define GSDR_TRK_SPL 8
#endif
constexpr int kSpl = GSDR_TRK_SPL;            // samples per lane per correlation chunk
constexpr int kWinCore = kSpl * kTrkThreads;  // 4096: the next call's window staged in LDS
constexpr int kHalo = 16;                     // slack around the predicted next start
constexpr int kStreamRow = 64 * 16;           // bytes one wave's global_load_lds_dwordx4 writes
constexpr int kCodeMargin = 32;              // replica samples copied on each side of the LDS replica
constexpr int kTimingSlots = 17;             // GSDR_TRK_TIMING record per call: 10 stamps + stream-wait ticks
                                             // + wave 2's lock test start / end and wave 0's
                                             // arrival at the join, wave 1's EVM end, wave 0 at the EVM
                                             // join and after it, as offsets from the partials barrier
constexpr int kStampSlots = 10;

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
// Galileo_E1.h:32-52
constexpr double kGalE1Hz = 1.57542e9;
constexpr double kGalE1Rate = 1.023e6;
constexpr double kGalE1Period = 0.004;
constexpr int kGalE1Length = 4092;
constexpr const char* kGalE1cSecondary = "0011100000001010110110010";
// Beidou_B1I.h:30-48
constexpr double kBdsB1Hz = 1.561098e9;
constexpr double kBdsB1Rate = 2.046e6;
constexpr double kBdsB1Period = 0.001;
constexpr int kBdsB1Length = 2046;
constexpr const char* kBdsB1Nh = "00000100110101001110";
constexpr const char* kBdsB1GeoPreamble = "1111110000001100001100";
constexpr const char* kGpsCaPreamble =
    "1111111111111111111100000000000000000000000000000000000000000000000000000000000011111111111111111111000000000000"
    "000000001111111111111111111111111111111111111111";
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

// Tracking_loop_filter::apply on a filter held in registers (wave 3's speculative
// DLL/PLL): the ring elements are separate scalars picked by selects -- with arrays
// the compiler turned the selects back into a run-time index, i.e. a scratch access
// (and the LDS form was a chain of dependent LDS round trips).  The reference's
// products and sums in its order.
struct LfReg
{
    float i0, i1, i2, i3, o0, o1, o2, o3, c0, c1, c2, c3, d0, d1, d2;
    int nin, nout, idx;
};

__device__ __forceinline__ LfReg lf_load(const LoopFilter& f)
{
    return LfReg{f.inputs[0], f.inputs[1], f.inputs[2], f.inputs[3], f.outputs[0], f.outputs[1], f.outputs[2],
        f.outputs[3], f.icoef[0], f.icoef[1], f.icoef[2], f.icoef[3], f.ocoef[0], f.ocoef[1], f.ocoef[2], f.nin, f.nout,
        f.idx};
}

__device__ __forceinline__ float lf_pick(float a0, float a1, float a2, float a3, int i)
{
    return i == 0 ? a0 : (i == 1 ? a1 : (i == 2 ? a2 : a3));
}

__device__ __forceinline__ float lf_apply(LfReg& f, float in)  // :58-93
{
    float r = 0.0F;
    const float oc[3] = {f.d0, f.d1, f.d2};
    const float ic[4] = {f.c0, f.c1, f.c2, f.c3};
#pragma unroll
    for (int ii = 0; ii < 3; ++ii)
        if (ii < f.nout) r += oc[ii] * lf_pick(f.o0, f.o1, f.o2, f.o3, (f.idx + ii) & 3);
    f.idx--;
    if (f.idx < 0) f.idx += 4;
    f.i0 = f.idx == 0 ? in : f.i0;
    f.i1 = f.idx == 1 ? in : f.i1;
    f.i2 = f.idx == 2 ? in : f.i2;
    f.i3 = f.idx == 3 ? in : f.i3;
#pragma unroll
    for (int ii = 0; ii < 4; ++ii)
        if (ii < f.nin) r += ic[ii] * lf_pick(f.i0, f.i1, f.i2, f.i3, (f.idx + ii) & 3);
    f.o0 = f.idx == 0 ? r : f.o0;
    f.o1 = f.idx == 1 ? r : f.o1;
    f.o2 = f.idx == 2 ? r : f.o2;
    f.o3 = f.idx == 3 ? r : f.o3;
    return r;
}

// Per-channel configuration: read-only inside the kernel (a separate restrict
// array, so its fields are fetched with scalar loads into SGPRs).
struct CfConst  // Tracking_FLL_PLL_filter coefficients
{
    float w0p3, w0f2, a2, w0f, a3, w0p2, b3, w0p;
    int order;
};

struct SmConst  // Exponential_Smoother parameters
{
    float alpha, one_minus_alpha, min_value, offset;
    int samples_init;
};

struct TrkConst
{
    double fs_in, code_period, code_chip_rate, signal_carrier_freq, carrier_lock_threshold;
    uint64_t acq_sample_stamp;
    uint64_t pull_in_span;   // (pull_in_time_s + 1) * (int)fs_in: the integer-second test of :1797 flips there
    uint64_t bit_sync_span;  // (bit_synchronization_time_limit_s + 1) * (int)fs_in (:1866)
    float early_late_space_chips;
    float shifts[kMaxTrkTaps];
    uint32_t preamble[5];    // secondary code / preamble as the circular-buffer register (acquire_secondary)
    uint32_t sec_str[5];     // secondary code string bit i = (code[i] == '1') (state-4 wipe-off)
    uint32_t data_sec_str;   // data secondary code (BeiDou NH), same form
    int32_t sec_len, data_sec_len, secondary, veml, track_pilot, iE, iP, iL;
    // extended coherent integration (state 3, :1945-1983): narrow taps, loops, time
    float shifts_narrow[kMaxTrkTaps];
    float early_late_space_narrow_chips, dll_bw_narrow_hz;
    double corr_time_ext;
    int32_t enable_ext;
    int32_t vector_length, code_length_chips, code_samples_per_chip, symbols_per_bit;
    int32_t cn0_samples, cn0_min, max_code_lock_fail, max_carrier_lock_fail;
    int32_t extend_correlation_symbols, enable_fll_pull_in, enable_fll_steady_state, carrier_aiding;
    int32_t n_taps, code_samples;
    uint32_t prn;
    CfConst cf;
    SmConst sm[2];  // 0: CN0, 1: carrier lock test
    CfConst cf_narrow;
    int32_t high_dyn, smoother_length;  // Dll_Pll_Conf::high_dyn / smoother_length (dll_pll_conf.h:62,80)
};

// Mutable scalar loop state (dll_pll_veml_tracking.h:117-209 minus the
// per-call temporaries): in wave 0's registers for a whole launch.
struct TrkHot
{
    double code_freq_chips, carrier_doppler_hz, acc_carrier_phase_rad, rem_code_phase_chips;
    double carrier_lock_test, cn0_db_hz, evm;
    double carrier_phase_step_rad, carrier_phase_rate_step_rad, code_phase_step_chips, code_phase_rate_step_chips;
    double rem_code_phase_samples;
    uint64_t next_sample;
    float2 VE_accu, E_accu, P_accu, P_accu_old, L_accu, VL_accu, P_data_accu;
    float cf_w, cf_x;                  // Tracking_FLL_PLL_filter state
    float sm_old[2], sm_sum[2];        // smoothers: value and running init sum
    int32_t sm_counter[2], sm_init[2];
    uint32_t circ[5];                  // signs of the last kPreambleLen prompts (1 = real < 0), newest at bit 0
    int32_t circ_size;
    float rem_carr_phase_rad, spc;
    int32_t state, current_prn_length_samples, current_symbol, current_data_symbol, cn0_estimation_counter;
    int32_t carrier_lock_fail_counter, code_lock_fail_counter;
    int32_t pull_in_transitory, cloop, acc_carrier_phase_initialized, flag_pll_180;
    double corr_time;            // d_current_correlation_time_s
    int32_t narrow, extend_count;  // after the switch to the extended correlator
    int32_t hist_n, hist_head;     // high_dyn: d_carr_ph_history / d_code_ph_history fill and oldest slot
    // run_dll_pll's d_carr_phase_error_hz, d_carr_error_filt_hz, d_code_error_chips,
    // d_code_error_filt_chips as log_data writes them (float of the double members)
    float log_err[4];
};

// Device-memory image of the mutable part of one channel.
struct TrkChan
{
    TrkHot h;
    LoopFilter code_filter;
    float2 prompt_buffer[kMaxCn0];
    // high_dyn: the two boost::circular_buffer<pair<double,double>> of capacity
    // 2*smoother_length (:554-563), pushed together (same sample count)
    double hist_carr[2 * kMaxSmoother], hist_code[2 * kMaxSmoother], hist_samples[2 * kMaxSmoother];
};

// The loop state make_prep reads (wave 0 -> wave 1 after the locked branch): wave 1 plans
// the next call while wave 0 takes the lock test and writes the record
struct PlanIn
{
    double carrier_phase_step_rad, carrier_phase_rate_step_rad, rem_code_phase_chips, code_phase_step_chips,
        code_phase_rate_step_chips;
    uint64_t next_sample;
    float rem_carr_phase_rad;
    int32_t state, narrow;
};

struct Prep  // lane-0 -> workgroup broadcast of one call's NCO
{
    double psi0, theta;
    float2 wstep;
    float rem_code, code_step;
    int64_t off;
    int32_t go;
    int32_t woff;  // >= 0: this call's samples are in the LDS window at that offset
    int32_t wrap;  // code index range of the call: 2 within the replica's margins, 1 within [-L, 2L), 0 general
    int32_t narrow;  // the call uses the narrow tap shifts
    int32_t pf_ok;   // streamed call: chunk 0 is in the buffer prefetched during the previous update
    // high_dyn: rotator rate term and resampler rate (do_correlation_step, :1069-1075),
    // taps 1..K-1 as sample-shifted copies of tap 0 (32f_xn_high_dynamics_resampler_32f_xn.h:84-91)
    int32_t hd;
    double theta_rate;
    float code_rate;
    int32_t hdshift[kMaxTrkTaps];
};

// ------------------------------------------------------------------ wave-0 loop body
// The loop update runs on all 64 lanes of wave 0 with identical (uniform)
// values; the loops over the CN0 buffer put one element on each lane and sum in
// the reference's element order with readlane, so results are bit-identical to
// the sequential code.  Memory writes are done by lane 0.
__device__ __forceinline__ float lane_f(float v, int i) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), i)); }

__device__ inline float cf_error(const CfConst& k, TrkHot& t, float fll, float pll, float tc)  // :77-101
{
    float e;
    if (k.order == 3)
        {
            t.cf_w = t.cf_w + tc * (k.w0p3 * pll + k.w0f2 * fll);
            t.cf_x = t.cf_x + tc * (0.5F * t.cf_w + k.a2 * k.w0f * fll + k.a3 * k.w0p2 * pll);
            e = 0.5F * t.cf_x + k.b3 * k.w0p * pll;
        }
    else
        {
            const float wn = t.cf_w + pll * k.w0p2 * tc + fll * k.w0f * tc;
            e = 0.5F * (wn + t.cf_w) + k.a2 * k.w0p * pll;
            t.cf_w = wn;
        }
    return e;
}

__device__ inline float sm_smooth(const SmConst& k, TrkHot& t, int w, float raw)  // exponential_smoother.cc:84-110
{
    float v;
    if (t.sm_init[w])
        {
            t.sm_counter[w]++;
            v = raw;
            t.sm_sum[w] = t.sm_sum[w] + v;
            if (t.sm_counter[w] == k.samples_init)
                {
                    t.sm_old[w] = t.sm_sum[w] / (float)t.sm_counter[w];
                    if (t.sm_old[w] < (k.min_value + k.offset))
                        {
                            t.sm_counter[w] = 0;
                            t.sm_sum[w] = 0.0F;
                        }
                    else
                        t.sm_init[w] = 0;
                }
        }
    else
        {
            v = k.alpha * raw + k.one_minus_alpha * t.sm_old[w];
            t.sm_old[w] = v;
        }
    return v;
}

__host__ __device__ inline void sm_reset(TrkHot& t, int w)
{
    t.sm_init[w] = 1;
    t.sm_counter[w] = 0;
    t.sm_sum[w] = 0.0F;
}

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

// pll_four_quadrant_atan (:86-89); gr::fast_atan2f restated as atan2f
__device__ inline double pll_four_quadrant_atan(float2 p) { return (double)atan2f(p.y, p.x); }

__device__ inline double dll_nc_vemlp(float2 ve, float2 e, float2 l, float2 vl)  // :139-149
{
    const double Early = sqrt((double)(ve.x * ve.x + ve.y * ve.y + e.x * e.x + e.y * e.y));
    const double Late = sqrt((double)(l.x * l.x + l.y * l.y + vl.x * vl.x + vl.y * vl.y));
    const double s = Early + Late;
    if (s == 0.0) return 0.0;
    return (Early - Late) / s;
}

__device__ inline void clear_tracking_vars(TrkHot& t)  // :1192-1213
{
    t.P_accu_old = make_float2(0.f, 0.f);
    t.current_symbol = 0;
    t.current_data_symbol = 0;
    t.circ_size = 0;
    for (int w = 0; w < 5; ++w) t.circ[w] = 0u;
    t.carrier_phase_rate_step_rad = 0.0;
    t.code_phase_rate_step_chips = 0.0;
    t.hist_n = 0;  // d_carr_ph_history.clear(), d_code_ph_history.clear()
    t.hist_head = 0;
    for (int i = 0; i < 4; ++i) t.log_err[i] = 0.0F;
}

// Sequential float sums over the buffer elements (the estimators' loops, in the
// reference's element order): every lane of wave 0 reads the per-element terms
// back from LDS (same address on all lanes) and adds them in order.
template <int NS>
__device__ __forceinline__ void seq_sums(const float* terms, int stride, int n, float (&sum)[NS])
{
    __builtin_amdgcn_wave_barrier();
    for (int q = 0; q < NS; ++q) sum[q] = 0.0F;
    int i = 0;
    for (; i + 4 <= n; i += 4)
        {
            float4 v[NS];
#pragma unroll
            for (int q = 0; q < NS; ++q) v[q] = *reinterpret_cast<const float4*>(terms + q * stride + i);
#pragma unroll
            for (int q = 0; q < NS; ++q) sum[q] += v[q].x;
#pragma unroll
            for (int q = 0; q < NS; ++q) sum[q] += v[q].y;
#pragma unroll
            for (int q = 0; q < NS; ++q) sum[q] += v[q].z;
#pragma unroll
            for (int q = 0; q < NS; ++q) sum[q] += v[q].w;
        }
    for (; i < n; ++i)
#pragma unroll
        for (int q = 0; q < NS; ++q) sum[q] += terms[q * stride + i];
}

// cn0_and_tracking_lock_status (:970-1056) with cn0_m2m4_estimator and
// carrier_lock_detector (lock_detectors.cc:90-148); wave 2 on its copy of the
// call's state (Cn0Spec), lane = element,
// sums in element order through `scratch` (3 x kMaxCn0 floats of LDS).  Returns 0 on a
// loss of lock, 1 while the prompt buffer fills, 2 with a full buffer: then the EVM
// (:1027-1053, an output only) is the one wave 1 computes (evm_of).
__device__ inline int cn0_and_lock(const TrkConst& c, TrkHot& t, float2* pbuf, float (*scratch)[kMaxCn0], double coh,
    int lane)
{
    const int n = c.cn0_samples;
    if (t.cn0_estimation_counter < n)
        {
            if (lane == 0) pbuf[t.cn0_estimation_counter] = t.P_accu;
            t.cn0_estimation_counter++;
            return 1;
        }
    const int widx = t.cn0_estimation_counter % n;
    float2 ei = make_float2(0.f, 0.f);
    if (lane < n) ei = lane == widx ? t.P_accu : pbuf[lane];
    if (lane == 0) pbuf[widx] = t.P_accu;
    t.cn0_estimation_counter++;
    // cn0_m2m4_estimator: Psig += |re|; aux = im*im + re*re; m2 += aux; m4 += aux*aux
    const float a_i = fabsf(ei.x);
    const float aux_i = ei.y * ei.y + ei.x * ei.x;
    const float aux2_i = aux_i * aux_i;
    scratch[0][lane] = a_i;
    scratch[1][lane] = aux_i;
    scratch[2][lane] = aux2_i;
    float sums[3];
    seq_sums<3>(&scratch[0][0], kMaxCn0, n, sums);
    float psig = sums[0], m2 = sums[1], m4 = sums[2];
    const float fn = (float)n;
    psig /= fn;
    psig = psig * psig;
    m2 /= fn;
    m4 /= fn;
    float aux = sqrtf(2.0F * m2 * m2 - m4);
    float snr;
    if (isnan(aux))
        snr = psig / (m2 - psig);
    else
        snr = aux / (m2 - aux);
    const float raw = 10.0F * log10f(snr) - 10.0F * log10f((float)coh);
    t.cn0_db_hz = (double)sm_smooth(c.sm[0], t, 0, raw);
    // carrier_lock_detector(buffer, 1): element 0 only
    const float si = 0.0F + lane_f(ei.x, 0), sq = 0.0F + lane_f(ei.y, 0);
    const float lock = (si * si - sq * sq) / (si * si + sq * sq);
    t.carrier_lock_test = (double)sm_smooth(c.sm[1], t, 1, lock);
    if (!t.pull_in_transitory)
        {
            if (t.carrier_lock_test < c.carrier_lock_threshold)
                t.carrier_lock_fail_counter++;
            else if (t.carrier_lock_fail_counter > 0)
                t.carrier_lock_fail_counter--;
            if (t.cn0_db_hz < c.cn0_min)
                t.code_lock_fail_counter++;
            else if (t.code_lock_fail_counter > 0)
                t.code_lock_fail_counter--;
        }
    if (t.carrier_lock_fail_counter > c.max_carrier_lock_fail || t.code_lock_fail_counter > c.max_code_lock_fail)
        {
            t.carrier_lock_fail_counter = 0;
            t.code_lock_fail_counter = 0;
            return 0;
        }
    return 2;
}

// The fork indicator EVM of cn0_and_tracking_lock_status (:1027-1053) on wave 1, from
// the prompt buffer with this call's prompt (a full buffer: cn0_estimation_counter >=
// cn0_samples before the call): the same float sums in element order as the oracle,
// through `scratch` (2 x kMaxCn0 floats of LDS).
__device__ inline double evm_of(const TrkConst& c, int cn0_counter, float2 p_accu, const float2* pbuf, float* scratch,
    int lane)
{
    const int n = c.cn0_samples;
    const int widx = cn0_counter % n;
    float2 ei = make_float2(0.f, 0.f);
    if (lane < n) ei = lane == widx ? p_accu : pbuf[lane];
    scratch[lane] = ei.x * ei.x;  // sum of squared in-phase prompts
    float s1[1];
    seq_sums<1>(scratch, 0, n, s1);
    const float fn = (float)n;
    float d = s1[0] / fn;
    d = sqrtf(d);
    const float ea = fabsf(ei.x / d) - 1.0F;
    const float eb = fabsf(ei.y / d) - 0.0F;
    const float aa_i = ea * ea, bb_i = eb * eb;
    __builtin_amdgcn_wave_barrier();
    scratch[2 * lane] = aa_i;  // interleaved: s = s + aa_i; s = s + bb_i in element order
    scratch[2 * lane + 1] = bb_i;
    float s2[1];
    seq_sums<1>(scratch, 0, 2 * n, s2);
    return sqrt((double)(s2[0] / fn / 1.0F));
}

// run_dll_pll (:1092-1179, no Doppler correction) as its two independent halves, on
// two waves: the carrier loop (PLL / FLL discriminators and filter) and the code loop
// (DLL discriminator and filter); the carrier aiding term, the one product of the two,
// is added where they are joined (take_dll_pll), in the reference's order
__device__ inline void run_pll(const TrkConst& c, TrkHot& t)
{
    const double carr_phase_error_hz =
        (t.cloop ? pll_cloop_two_quadrant_atan(t.P_accu) : pll_four_quadrant_atan(t.P_accu)) / kTwoPi;
    double carr_error_filt_hz;
    if ((t.pull_in_transitory && c.enable_fll_pull_in) || c.enable_fll_steady_state)
        {
            const double carr_freq_error_hz = fll_diff_atan(t.P_accu_old, t.P_accu, 0, t.corr_time) / kTwoPi;
            t.P_accu_old = t.P_accu;
            if (t.pull_in_transitory && c.enable_fll_pull_in)
                carr_error_filt_hz = (double)cf_error(t.narrow ? c.cf_narrow : c.cf, t, (float)carr_freq_error_hz, 0.0F,
                    (float)t.corr_time);
            else
                carr_error_filt_hz = (double)cf_error(t.narrow ? c.cf_narrow : c.cf, t, (float)carr_freq_error_hz, (float)carr_phase_error_hz,
                    (float)t.corr_time);
        }
    else
        {
            carr_error_filt_hz = (double)cf_error(t.narrow ? c.cf_narrow : c.cf, t, 0, (float)carr_phase_error_hz, (float)t.corr_time);
        }
    t.carrier_doppler_hz = carr_error_filt_hz;
    t.log_err[0] = (float)carr_phase_error_hz;
    t.log_err[1] = (float)carr_error_filt_hz;
}

// the code loop's d_code_freq_chips before the carrier aiding term
__device__ inline double run_dll(const TrkConst& c, TrkHot& t, LfReg& lf)
{
    const double code_error_chips =
        c.veml ? dll_nc_vemlp(t.VE_accu, t.E_accu, t.L_accu, t.VL_accu) : dll_nc_e_minus_l(t.E_accu, t.L_accu, t.spc, 1.0F, 1.0F);
    const double code_error_filt_chips = (double)lf_apply(lf, (float)code_error_chips);
    t.log_err[2] = (float)code_error_chips;
    t.log_err[3] = (float)code_error_filt_chips;
    return c.code_chip_rate - code_error_filt_chips;
}

// high_dyn rate estimate (:1232-1251, :1265-1284): mean of the newest
// smoother_length steps minus mean of the oldest, over the newest sample counts,
// summed in the reference's order ([k] counts from the oldest element).  The
// element just pushed (slot) comes from registers, not read back.
__device__ inline double hist_rate(const double* v, const double* s, int head, int cap, int L, int slot, double vnew,
    double snew)
{
    double cp1 = 0.0, cp2 = 0.0, samples = 0.0;
    for (int k = 0; k < L; ++k)
        {
            const int a = (head + k) % cap, b = (head + 2 * L - k - 1) % cap;
            cp1 += a == slot ? vnew : v[a];
            cp2 += b == slot ? vnew : v[b];
            samples += b == slot ? snew : s[b];
        }
    cp1 /= (double)L;
    cp2 /= (double)L;
    return (cp2 - cp1) / samples;
}

// Every lane of wave 0 runs this with uniform values; the history stores write
// the same value from every lane.
__device__ inline void update_tracking_vars(const TrkConst& c, TrkHot& t, TrkChan* gc)  // :1216-1287
{
    const double T_chip = 1.0 / t.code_freq_chips;
    const double T_prn = T_chip * (double)c.code_length_chips;
    const double T_prn_samples = T_prn * c.fs_in;
    const double K_blk = T_prn_samples + t.rem_code_phase_samples;
    t.current_prn_length_samples = (int32_t)floor(K_blk);
    t.carrier_phase_step_rad = kTwoPi * t.carrier_doppler_hz / c.fs_in;
    int slot = 0;
    const int cap = 2 * c.smoother_length;
    const double ns = (double)t.current_prn_length_samples;
    if (c.high_dyn)
        {
            // push_back on a full circular buffer overwrites the oldest element
            if (t.hist_n < cap)
                {
                    slot = (t.hist_head + t.hist_n) % cap;
                    t.hist_n++;
                }
            else
                {
                    slot = t.hist_head;
                    t.hist_head = (t.hist_head + 1) % cap;
                }
            if (t.hist_n == cap)
                t.carrier_phase_rate_step_rad = hist_rate(gc->hist_carr, gc->hist_samples, t.hist_head, cap,
                    c.smoother_length, slot, t.carrier_phase_step_rad, ns);
            gc->hist_carr[slot] = t.carrier_phase_step_rad;
        }
    const double len = (double)t.current_prn_length_samples;
    t.rem_carr_phase_rad += (float)(t.carrier_phase_step_rad * len + 0.5 * t.carrier_phase_rate_step_rad * len * len);
    t.rem_carr_phase_rad = (float)fmod((double)t.rem_carr_phase_rad, kTwoPi);
    t.acc_carrier_phase_rad -= (t.carrier_phase_step_rad * len + 0.5 * t.carrier_phase_rate_step_rad * len * len);
    t.code_phase_step_chips = t.code_freq_chips / c.fs_in;
    if (c.high_dyn)
        {
            if (t.hist_n == cap)
                t.code_phase_rate_step_chips = hist_rate(gc->hist_code, gc->hist_samples, t.hist_head, cap,
                    c.smoother_length, slot, t.code_phase_step_chips, ns);
            gc->hist_code[slot] = t.code_phase_step_chips;
            gc->hist_samples[slot] = ns;
        }
    t.rem_code_phase_samples = K_blk - len;
    t.rem_code_phase_chips = t.code_freq_chips * t.rem_code_phase_samples / c.fs_in;
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
    t.circ_size++;
}

// acquire_secondary (:923-967): corr = sum over the buffer of +-1 by sign match
// = 160 - 2 * mismatches; |corr| == 160 only on a full match or full inversion.
__device__ inline int acquire_secondary(const TrkConst& c, TrkHot& t)
{
    // the last sec_len pushes sit in register bits [0, sec_len)
    int mism = 0;
    for (int w = 0; w < 5; ++w)
        {
            const int lo = w * 32;
            const uint32_t mask = c.sec_len >= lo + 32 ? 0xffffffffu : (c.sec_len > lo ? (1u << (c.sec_len - lo)) - 1u : 0u);
            mism += __popc((t.circ[w] ^ c.preamble[w]) & mask);
        }
    if (mism == 0)
        {
            t.flag_pll_180 = 0;
            return 1;
        }
    if (mism == c.sec_len)
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
    float log_accu[5];  // log_data's |VE|, |E|, |P|, |L|, |VL| accumulators (GSDR_TRK_F_LOGGED)
    bool evm;           // locked with a full prompt buffer: t.evm is wave 1's evm_of
};

// log_data (:1403-1500): the accumulator magnitudes at the reference's log point
// (std::abs<float> of the complex accumulators; VE/VL written as 0 without VEML)
__device__ inline void log_point(const TrkConst& c, const TrkHot& t, EpochOut& o)
{
    o.flags |= GSDR_TRK_F_LOGGED;
    o.log_accu[0] = c.veml ? hypotf(t.VE_accu.x, t.VE_accu.y) : 0.0F;
    o.log_accu[1] = hypotf(t.E_accu.x, t.E_accu.y);
    o.log_accu[2] = hypotf(t.P_accu.x, t.P_accu.y);
    o.log_accu[3] = hypotf(t.L_accu.x, t.L_accu.y);
    o.log_accu[4] = c.veml ? hypotf(t.VL_accu.x, t.VL_accu.y) : 0.0F;
}

// save_correlation_results (:1288-1400): secondary-code wipe-off of the tap
// accumulators, data-symbol accumulation (NH wipe-off / pilot data prompt).
// epl: the taps at c.iE / c.iP / c.iL (summed from LDS by run-time index, so no
// private array is indexed at run time)
__device__ inline void save_correlation_results(const TrkConst& c, TrkHot& t, const float2 (&taps)[kMaxTrkTaps + 1],
    const float2 (&epl)[3])
{
    float sg = 1.0F;
    if (c.secondary)
        {
            sg = ((c.sec_str[t.current_symbol >> 5] >> (t.current_symbol & 31)) & 1u) ? -1.0F : 1.0F;
            t.current_symbol++;
            t.current_symbol %= c.sec_len;
        }
    auto acc = [](float2& a, float2 b, float g) {
        if (g > 0)
            {
                a.x += b.x;
                a.y += b.y;
            }
        else
            {
                a.x -= b.x;
                a.y -= b.y;
            }
    };
    if (c.veml)
        {
            acc(t.VE_accu, taps[0], sg);
            acc(t.VL_accu, taps[4], sg);
        }
    acc(t.E_accu, epl[0], sg);
    acc(t.P_accu, epl[1], sg);
    acc(t.L_accu, epl[2], sg);
    const float2 pd = c.track_pilot ? taps[kMaxTrkTaps] : epl[1];
    if (c.symbols_per_bit > 1)
        {
            if (c.data_sec_len > 0)
                {
                    acc(t.P_data_accu, pd, ((c.data_sec_str >> t.current_data_symbol) & 1u) ? -1.0F : 1.0F);
                    t.current_data_symbol++;
                    t.current_data_symbol %= c.data_sec_len;
                }
            else
                {
                    acc(t.P_data_accu, pd, 1.0F);
                    t.current_data_symbol++;
                    t.current_data_symbol %= c.symbols_per_bit;
                }
        }
    else
        t.P_data_accu = pd;
    t.cloop = c.track_pilot ? 0 : 1;
}

// One general_work call after the correlation (taps given; slot kMaxTrkTaps is
// the pilot-tracking data prompt): states 2 and 4.
// GSDR_TRK_TIMING: wall-clock probes inside the loop update (slots 4-6 of the record)
__device__ __forceinline__ void tprobe(bool on, uint64_t (&pr)[3], int i)
{
    if (on) pr[i] = wall_clock64();
}

// run_dll_pll of a call computed speculatively (states 2 and 4) as its two halves:
// the carrier loop on wave 1, the code loop on wave 3 (into the code loop filter slot
// that is not current).  The discriminators and loop filters read nothing the CN0
// estimator and lock detector (wave 2) write, so each wave runs on its own copy of
// the state; wave 0 takes the results when the call stays locked (and drops them on a
// loss of lock).  Same operations on the same values: the loop is bit-identical to
// run_dll_pll on one wave (round 6: C2 call 6.2 -> 5.6 us, C5 GPS 10.8 -> 10.1 us,
// profiles/r06k3; with the next call's plan on wave 1 C5 GPS 9.9 us, profiles/r06p).
struct DllPllSpec  // wave 1's carrier loop of a call
{
    double carrier_doppler_hz;
    float2 P_accu_old;
    float cf_w, cf_x;
    float log_err[2];
};

// cn0_and_tracking_lock_status of a call computed by wave 2 (states 2 and 4): the
// fields it writes are disjoint from everything run_dll_pll, update_tracking_vars and
// the state transitions read or write, so wave 0 runs the locked branch without it and
// takes these results afterwards; on a loss of lock (rare) it rebuilds the call from
// the state at the call's start (s_t) exactly as the reference's early return leaves it.
struct Cn0Spec
{
    double cn0_db_hz, carrier_lock_test;
    float sm_old[2], sm_sum[2];
    int32_t sm_counter[2], sm_init[2];
    int32_t cn0_estimation_counter, carrier_lock_fail_counter, code_lock_fail_counter, locked;
};

__device__ __forceinline__ void cn0_publish(Cn0Spec& r, const TrkHot& t, int locked)
{
    r.cn0_db_hz = t.cn0_db_hz;
    r.carrier_lock_test = t.carrier_lock_test;
    for (int w = 0; w < 2; ++w)
        {
            r.sm_old[w] = t.sm_old[w];
            r.sm_sum[w] = t.sm_sum[w];
            r.sm_counter[w] = t.sm_counter[w];
            r.sm_init[w] = t.sm_init[w];
        }
    r.cn0_estimation_counter = t.cn0_estimation_counter;
    r.carrier_lock_fail_counter = t.carrier_lock_fail_counter;
    r.code_lock_fail_counter = t.code_lock_fail_counter;
    r.locked = locked;
}

__device__ __forceinline__ void cn0_apply(TrkHot& t, const Cn0Spec& r)
{
    t.cn0_db_hz = r.cn0_db_hz;
    t.carrier_lock_test = r.carrier_lock_test;
    for (int w = 0; w < 2; ++w)
        {
            t.sm_old[w] = r.sm_old[w];
            t.sm_sum[w] = r.sm_sum[w];
            t.sm_counter[w] = r.sm_counter[w];
            t.sm_init[w] = r.sm_init[w];
        }
    t.cn0_estimation_counter = r.cn0_estimation_counter;
    t.carrier_lock_fail_counter = r.carrier_lock_fail_counter;
    t.code_lock_fail_counter = r.code_lock_fail_counter;
}

struct DllSpec  // wave 3's code loop of a call
{
    double code_freq_base;  // c.code_chip_rate - the filtered code error
    float log_err2, log_err3;
};

struct SpecLink
{
    DllPllSpec* res;   // LDS
    DllSpec* dres;     // LDS
    int* dready;       // LDS: the call index whose code loop dres holds
    int* ready;        // LDS: the call index whose results res holds
    LoopFilter* lfs;   // LDS: the code loop filter's two slots
    int* lfi_lds;      // LDS: the current slot (read by wave 3 at the start of a call)
    int lfi;           // wave 0: the current slot
    int e;             // wave 0: this call's index
};

__device__ inline void take_dll_pll(const TrkConst& c, TrkHot& t, SpecLink& sl)
{
    while (__hip_atomic_load(sl.ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != sl.e)
        __builtin_amdgcn_s_sleep(1);
    const DllPllSpec r = *sl.res;
    t.carrier_doppler_hz = r.carrier_doppler_hz;
    t.P_accu_old = r.P_accu_old;
    t.cf_w = r.cf_w;
    t.cf_x = r.cf_x;
    t.log_err[0] = r.log_err[0];
    t.log_err[1] = r.log_err[1];
    while (__hip_atomic_load(sl.dready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != sl.e)
        __builtin_amdgcn_s_sleep(1);
    const DllSpec d = *sl.dres;
    t.code_freq_chips = d.code_freq_base;
    t.log_err[2] = d.log_err2;
    t.log_err[3] = d.log_err3;
    if (c.carrier_aiding) t.code_freq_chips += t.carrier_doppler_hz * c.code_chip_rate / c.signal_carrier_freq;
    sl.lfi ^= 1;  // wave 3 filtered into the other slot
}

// The call's accumulators before the lock test (states 2 and 4, :1828-1845 / :2032):
// shared by wave 2's lock test, wave 0's locked branch and its rebuild after a loss
__device__ __forceinline__ void pre_lock(const TrkConst& c, TrkHot& t, const float2 (&taps)[kMaxTrkTaps + 1],
    const float2 (&epl)[3], uint64_t nitems_read)
{
    if (t.state == 2)
        {
            if (c.veml)
                {
                    t.VE_accu = taps[0];
                    t.VL_accu = taps[4];
                }
            t.E_accu = epl[0];
            t.P_accu = epl[1];
            t.L_accu = epl[2];
            t.spc = c.early_late_space_chips;
            if (nitems_read < c.acq_sample_stamp || nitems_read - c.acq_sample_stamp >= c.bit_sync_span)
                t.carrier_lock_fail_counter = 300000;
        }
    else
        save_correlation_results(c, t, taps, epl);
}

__device__ __forceinline__ void init_out(EpochOut& o)
{
    o.flags = 0;
    o.evm = false;
    o.prompt_i = 0.0;
    o.prompt_q = 0.0;
    for (int i = 0; i < 5; ++i) o.log_accu[i] = 0.0F;
}

// States 2 and 4 run the branch of a call that stays locked; the lock test's results
// come from wave 2 (Cn0Spec) and the caller undoes the branch on a loss of lock.
__device__ inline void after_correlation(const TrkConst& c, TrkHot& t, TrkChan* gc, SpecLink& sl,
    const float2 (&taps)[kMaxTrkTaps + 1], const float2 (&epl)[3], uint64_t nitems_read, EpochOut& o, bool tm,
    uint64_t (&pr)[3])
{
    init_out(o);
    if (t.state == 2)
        {
            pre_lock(c, t, taps, epl, nitems_read);
            tprobe(tm, pr, 0);
                {
                    int next_state = 0;
                    take_dll_pll(c, t, sl);
                    tprobe(tm, pr, 1);
                    update_tracking_vars(c, t, gc);
                    tprobe(tm, pr, 2);
                    log_point(c, t, o);
                    if (!t.pull_in_transitory)
                        {
                            if (c.secondary || c.symbols_per_bit > 1)
                                {
                                    circ_push(t, epl[1]);
                                    if (t.circ_size >= c.sec_len) next_state = acquire_secondary(c, t);
                                }
                            else
                                next_state = 1;
                        }
                    if (next_state)
                        {
                            t.VE_accu = t.E_accu = t.P_accu = t.L_accu = t.VL_accu = t.P_data_accu = make_float2(0.f, 0.f);
                            t.circ_size = 0;
                            for (int w = 0; w < 5; ++w) t.circ[w] = 0u;
                            t.current_symbol = 0;
                            t.current_data_symbol = 0;
                            o.flags |= GSDR_TRK_F_BIT_SYNC;
                            if (c.enable_ext)
                                {
                                    // extended correlator: narrow loops and taps (:1945-1983)
                                    t.extend_count = 0;
                                    t.corr_time = c.corr_time_ext;
                                    t.state = 3;
                                    LoopFilter& lf = sl.lfs[sl.lfi];
                                    lf.T = (float)t.corr_time;
                                    lf_update(lf);
                                    lf.bw = c.dll_bw_narrow_hz;
                                    lf_update(lf);
                                    t.narrow = 1;
                                    t.spc = c.early_late_space_narrow_chips;
                                }
                            else
                                t.state = 4;
                        }
                }
        }
    else if (t.state == 3)  // coherent integration (:1989-2026)
        {
            save_correlation_results(c, t, taps, epl);
            update_tracking_vars(c, t, gc);
            if (t.current_data_symbol == 0)
                {
                    log_point(c, t, o);
                    o.prompt_i = (double)t.P_data_accu.x;
                    o.prompt_q = (double)t.P_data_accu.y;
                    o.flags |= GSDR_TRK_F_VALID_OUTPUT;
                    t.P_data_accu = make_float2(0.f, 0.f);
                }
            t.extend_count++;
            if (t.extend_count == c.extend_correlation_symbols - 1)
                {
                    t.extend_count = 0;
                    t.state = 4;
                }
        }
    else  // state 4
        {
            pre_lock(c, t, taps, epl, nitems_read);
            tprobe(tm, pr, 0);
                {
                    take_dll_pll(c, t, sl);
                    tprobe(tm, pr, 1);
                    update_tracking_vars(c, t, gc);
                    tprobe(tm, pr, 2);
                    if (!t.acc_carrier_phase_initialized)
                        {
                            t.acc_carrier_phase_rad = -(double)t.rem_carr_phase_rad;
                            t.acc_carrier_phase_initialized = 1;
                        }
                    if (t.current_data_symbol == 0)
                        {
                            log_point(c, t, o);
                            o.prompt_i = (double)t.P_data_accu.x;
                            o.prompt_q = (double)t.P_data_accu.y;
                            o.flags |= GSDR_TRK_F_VALID_OUTPUT;
                            t.P_data_accu = make_float2(0.f, 0.f);
                        }
                    t.VE_accu = t.E_accu = t.P_accu = t.L_accu = t.VL_accu = make_float2(0.f, 0.f);
                    if (c.enable_ext) t.state = 3;
                }
        }
    if (t.flag_pll_180) o.flags |= GSDR_TRK_F_PLL_180;
}

template <int IT>
__device__ __forceinline__ float2 load_iq(const void* __restrict__ p, int64_t i)
{
    if constexpr (IT == GSDR_ITEM_GR_COMPLEX)
        return reinterpret_cast<const float2*>(p)[i];
    else if constexpr (IT == GSDR_ITEM_CSHORT)
        {
            const short2 s = reinterpret_cast<const short2*>(p)[i];
            return make_float2((float)s.x, (float)s.y);
        }
    else
        {
            // Ibyte_To_Complex: interleaved_char_to_complex, scale 1 (exact)
            const char2 s = reinterpret_cast<const char2*>(p)[i];
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

template <int IT>
constexpr int item_bytes()
{
    return IT == GSDR_ITEM_GR_COMPLEX ? 8 : (IT == GSDR_ITEM_CSHORT ? 4 : 2);
}

// one stream item from an LDS byte image of the input (raw item format)
template <int IT>
__device__ __forceinline__ float2 lds_iq(const char* b, int byte)
{
    if constexpr (IT == GSDR_ITEM_GR_COMPLEX)
        return *reinterpret_cast<const float2*>(b + byte);
    else if constexpr (IT == GSDR_ITEM_CSHORT)
        {
            const short2 v = *reinterpret_cast<const short2*>(b + byte);
            return make_float2((float)v.x, (float)v.y);
        }
    else
        {
            const char2 v = *reinterpret_cast<const char2*>(b + byte);
            return make_float2((float)v.x, (float)v.y);
        }
}

// Asynchronous copy of input bytes [first, first + nbytes) (relative to the
// stream pointer) into an LDS buffer with global_load_lds_dwordx4: no VGPR
// destinations, so a whole chunk is in flight at once.  The buffer starts at the
// 16-byte block holding `first` (returned); every lane's source is clamped to a
// 16-byte block holding at least one byte of the stream, i.e. inside the
// stream's own pages.  Waves [w0, kTrkThreads/64) issue; the buffer is valid
// after the issuing waves' vmcnt drains: each issuing wave runs s_waitcnt
// vmcnt(0) before the barrier that hands the buffer over (correlate_call_stream).
__device__ __forceinline__ uintptr_t stream_fetch(const void* iq, uint64_t iq_bytes, int64_t first, int nbytes,
    char* lds, int w0)
{
    const uintptr_t base = reinterpret_cast<uintptr_t>(iq);
    const uintptr_t lo = base & ~(uintptr_t)15;
    const uintptr_t hi = (base + iq_bytes - 1) & ~(uintptr_t)15;
    const uintptr_t start = (uintptr_t)((int64_t)base + first) & ~(uintptr_t)15;
    const int rows = (nbytes + 15 + kStreamRow - 1) / kStreamRow;  // first - start <= 15
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    for (int r = wave - w0; r < rows; r += kTrkThreads / 64 - w0)
        {
            if (r < 0) break;
            uintptr_t a = start + (uintptr_t)r * kStreamRow + (uintptr_t)lane * 16;
            a = a < lo ? lo : (a > hi ? hi : a);
            __builtin_amdgcn_global_load_lds((gsdr_gvoid*)a, (gsdr_lvoid*)(lds + r * kStreamRow), 16, 0, 0);
        }
    return start;
}

// (int)floorf(x) in one instruction (v_cvt_flr_i32_f32: floor, then convert; exact)
__device__ __forceinline__ int floor_i(float x)
{
    int r;
    asm("v_cvt_flr_i32_f32 %0, %1" : "=v"(r) : "v"(x));
    return r;
}

// The plan values every chunk of a call uses, in SGPRs: read from the LDS plan once
// per call.  Read per chunk, behind the streamed calls' barriers, their wait also
// waited for the chunk's own sample loads.
struct ChunkNco
{
    float cstep, wsx, wsy;
    int wrap;
};
__device__ __forceinline__ float uniform_f(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }
__device__ __forceinline__ ChunkNco chunk_nco(const Prep& p)
{
    return ChunkNco{uniform_f(p.code_step), uniform_f(p.wstep.x), uniform_f(p.wstep.y),
        __builtin_amdgcn_readfirstlane(p.wrap)};
}

// One correlation chunk of SPL (<= kSpl) samples per lane (n = n0 + tid +
// j*kTrkThreads), KT taps, no branches inside.  FULL: every sample of the chunk lies inside the
// call; otherwise samples past the end are zero and their index clamped.
// WRAP: 2 = every code index of the call lies in [-kCodeMargin, L + kCodeMargin),
// read straight from the margin-padded replica; 1 = in [-L, 2L), one conditional
// add/sub; 0 = general modulo.  Complex products and the accumulations are
// packed-f32 (v_pk_mul/v_pk_fma: one instruction per tap and sample).
// DATA: one more accumulator, acc[kMaxTrkTaps], on the data-component replica
// s_data at the prompt tap's index (the pilot-tracking data correlator of
// do_correlation_step, whose only tap sits at the prompt shift).
template <int IT, int SRC, int WRAP, bool FULL, int KT, bool DATA, int SPL = kSpl>
__device__ __forceinline__ void correlate_chunk(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const float* s_data, const Prep& p, const ChunkNco& q, int n0, int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph,
    float2 (&acc)[kMaxTrkTaps + 1], const char* sbuf = nullptr, int sboff = 0)
{
    using gsdr::pk::c2;
    constexpr int IPK = KT / 2;  // prompt slot: 1 of E,P,L / 2 of VE,E,P,L,VL
    // Five phases, fenced so the scheduler keeps them apart: (1) the samples (LDS
    // or HBM) go out first -- left alone the scheduler sank their reads below the
    // replica gathers, each behind its own lgkmcnt(0), four serial LDS round trips
    // per chunk; (2) every replica index; (3) every replica gather (the data
    // replica's first, at the prompt indices), then tap-major; (4) the rotated samples (the phasor
    // chain, under the gathers' latency); (5) the FMAs tap-major, so each tap's
    // FMAs wait only for that tap's gathers.  Every accumulator still adds its
    // samples in increasing j, so the sums are those of the sample-major order.
    const float cstep = q.cstep;
    const c2 ws = c2{q.wsx, q.wsy};
    c2 xs[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j)
        {
            const int n = n0 + (int)threadIdx.x + j * kTrkThreads;
            const int nc = FULL ? n : min(n, vl - 1);
            float2 v;
            if constexpr (SRC == 0)
                v = s_win[p.woff + nc];
            else if constexpr (SRC == 1)
                v = load_iq<IT>(iq, p.off + nc);
            else
                v = lds_iq<IT>(sbuf, sboff + nc * item_bytes<IT>());
            xs[j] = gsdr::pk::from(v);  // masked in phase 4: a select here waits for the load
        }
    __builtin_amdgcn_sched_barrier(0);
    float cv[SPL][KT];
    float dv[SPL];
#pragma unroll
    for (int j = 0; j < SPL; ++j)
        {
            const int n0j = n0 + (int)threadIdx.x + j * kTrkThreads;
            const int n = FULL ? n0j : min(n0j, vl - 1);
            const float a = gsdr::mul_rn(cstep, (float)n);
#pragma unroll
            for (int k = 0; k < KT; ++k)
                {
                    // a_avx association: floor(step*n + (shift - rem))
                    int raw = floor_i(gsdr::add_rn(a, sh_rem[k]));
                    if (WRAP == 1)
                        {
                            raw += raw < 0 ? L : 0;
                            raw -= raw >= L ? L : 0;
                        }
                    else if (WRAP == 0)
                        raw = wrap_code(raw, L);
                    cv[j][k] = __int_as_float(raw);
                }
        }
    if (DATA)
        {
            // first: the data replica is gathered at the prompt tap's index
#pragma unroll
            for (int j = 0; j < SPL; ++j) dv[j] = s_data[__float_as_int(cv[j][IPK])];
        }
#pragma unroll
    for (int k = 0; k < KT; ++k)
        {
#pragma unroll
            for (int j = 0; j < SPL; ++j) cv[j][k] = s_code[__float_as_int(cv[j][k])];
        }
    __builtin_amdgcn_sched_barrier(0);
    c2 tt[SPL];
    c2 phv = gsdr::pk::from(ph);
#pragma unroll
    for (int j = 0; j < SPL; ++j)
        {
            if (!FULL && n0 + (int)threadIdx.x + j * kTrkThreads >= vl) xs[j] = c2{0.f, 0.f};
            tt[j] = gsdr::pk::mul(xs[j], phv);
            phv = gsdr::pk::mul(phv, ws);
        }
    ph = gsdr::pk::to(phv);
#pragma unroll
    for (int k = 0; k < KT; ++k)
        {
            c2 av = gsdr::pk::from(acc[k]);
#pragma unroll
            for (int j = 0; j < SPL; ++j) av = gsdr::pk::fmas(tt[j], cv[j][k], av);
            acc[k] = gsdr::pk::to(av);
        }
    if (DATA)
        {
            c2 av = gsdr::pk::from(acc[kMaxTrkTaps]);
#pragma unroll
            for (int j = 0; j < SPL; ++j) av = gsdr::pk::fmas(tt[j], dv[j], av);
            acc[kMaxTrkTaps] = gsdr::pk::to(av);
        }
}

// the chunk at n0 with the call's wrap mode; FULL when the whole chunk is inside the call
template <int IT, int SRC, int KT, bool DATA, int SPL>
__device__ __forceinline__ void correlate_chunk_wrap(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const float* s_data, const Prep& p, const ChunkNco& q, int n0, int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph,
    float2 (&acc)[kMaxTrkTaps + 1], const char* sbuf, int sboff)
{
    if (q.wrap == 2)
        {
            if (SPL == kSpl && n0 + kWinCore <= vl)
                correlate_chunk<IT, SRC, 2, true, KT, DATA, SPL>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc,
                    sbuf, sboff);
            else
                correlate_chunk<IT, SRC, 2, false, KT, DATA, SPL>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc,
                    sbuf, sboff);
        }
    else if (q.wrap == 1)
        correlate_chunk<IT, SRC, 1, false, KT, DATA, SPL>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc, sbuf,
            sboff);
    else
        correlate_chunk<IT, SRC, 0, false, KT, DATA, SPL>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc, sbuf,
            sboff);
}

// A call's last chunk that holds fewer than kWinCore samples runs with as few
// samples per lane as cover it (1, 2, 4 or kSpl): a 25000-sample call's last 424
// samples take one sample per lane instead of a full chunk of masked ones.  The
// samples and their order are those of the full chunk (a masked sample adds 0).
template <int IT, int SRC, int KT, bool DATA>
__device__ __forceinline__ void correlate_chunk_any(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const float* s_data, const Prep& p, const ChunkNco& q, int n0, int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph,
    float2 (&acc)[kMaxTrkTaps + 1], const char* sbuf = nullptr, int sboff = 0)
{
    const int rest = vl - n0;
    if (rest >= kWinCore || rest > 4 * kTrkThreads || kSpl <= 4)
        correlate_chunk_wrap<IT, SRC, KT, DATA, kSpl>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc, sbuf, sboff);
    else if (rest > 2 * kTrkThreads)
        correlate_chunk_wrap<IT, SRC, KT, DATA, 4>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc, sbuf, sboff);
    else if (rest > kTrkThreads)
        correlate_chunk_wrap<IT, SRC, KT, DATA, 2>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc, sbuf, sboff);
    else
        correlate_chunk_wrap<IT, SRC, KT, DATA, 1>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc, sbuf, sboff);
}

// high_dyn correlation (do_correlation_step with set_high_dynamics_resampler(true)):
// VOLK-GNSSSDR 32f_xn_high_dynamics_resampler_32f_xn generic (:67-96: tap 0 index
// floor(step*m + rate*(m*m) + shift0 - rem) with the unsigned m*m, taps 1..K-1 the
// sample-shifted copies of tap 0) and 32fc_32f_high_dynamic_rotator_dot_prod_32fc_xn
// (:68-112: sample n rotated by the phase of n*theta + (n-1)^2*theta_rate, from the
// fp64 model as in corr.hip).  Lane-strided samples; the window or HBM as the fast path.
// (always inlined: as a call it took the address of the kernel's accumulators,
// which then lived in scratch for every correlation path)
template <int IT>
__device__ __forceinline__ void correlate_call_hd(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const float* s_data, const Prep& p, int vl, int L, int K, bool data, float shift0, float shiftP,
    float2 (&acc)[kMaxTrkTaps + 1])
{
    constexpr double kInvTwoPi = 0.15915494309189533576888376337251;
    auto index = [&](float shift, uint32_t m) {
        const float a = gsdr::mul_rn(p.code_step, (float)m);
        const float b = gsdr::mul_rn(p.code_rate, (float)(m * m));
        int raw = (int)floorf(gsdr::sub_rn(gsdr::add_rn(gsdr::add_rn(a, b), shift), p.rem_code));
        raw %= L;
        return raw < 0 ? raw + L : raw;
    };
    for (int n = (int)threadIdx.x; n < vl; n += kTrkThreads)
        {
            const float2 x = p.woff >= 0 ? s_win[p.woff + n] : load_iq<IT>(iq, p.off + n);
            double phi = p.psi0 + (double)n * p.theta;
            if (n > 0)
                {
                    const double m1 = (double)(n - 1);
                    phi += m1 * m1 * p.theta_rate;
                }
            const float ang = (float)fma(-rint(phi * kInvTwoPi), kTwoPi, phi);
            float sn, cs;
            sincosf(ang, &sn, &cs);
            const float2 tt = make_float2(x.x * cs - x.y * sn, x.x * sn + x.y * cs);
#pragma unroll
            for (int k = 0; k < kMaxTrkTaps; ++k)
                {
                    if (k < K)
                        {
                            const float cv = s_code[index(shift0, (uint32_t)((n + p.hdshift[k]) % vl))];
                            acc[k].x += tt.x * cv;
                            acc[k].y += tt.y * cv;
                        }
                }
            if (data)
                {
                    const float dv = s_data[index(shiftP, (uint32_t)n)];
                    acc[kMaxTrkTaps].x += tt.x * dv;
                    acc[kMaxTrkTaps].y += tt.y * dv;
                }
        }
}

template <int IT, int KT, bool DATA>
__device__ __forceinline__ void correlate_call(const void* __restrict__ iq, const float2* s_win, const float* s_code,
    const float* s_data, const Prep& p, int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph,
    float2 (&acc)[kMaxTrkTaps + 1])
{
    const ChunkNco q = chunk_nco(p);
    for (int n0 = 0; n0 < vl; n0 += kWinCore)
        {
            if (p.woff >= 0)
                correlate_chunk_any<IT, 0, KT, DATA>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc);
            else
                correlate_chunk_any<IT, 1, KT, DATA>(iq, s_win, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc);
        }
}

// Streamed call (vector_length > kWinCore): the call's samples pass through two
// LDS chunk buffers of `chunk` samples filled by global_load_lds.  Chunk j is
// read from buffer j&1 while chunk j+1 lands in the other; chunk 0 was
// prefetched during the previous call's loop update when `pf_ok` (else fetched
// here).  The __syncthreads at the top of each chunk drains the DMA (vmcnt(0))
// and orders the previous chunk's reads before its buffer is refilled.
template <int IT, int KT, bool DATA>
__device__ __forceinline__ void correlate_call_stream(const void* __restrict__ iq, uint64_t iq_items, char* sb,
    int sbuf_bytes, int chunk, bool pf_ok, const uintptr_t (&pf_start)[2], const float* s_code, const float* s_data, const Prep& p,
    int vl, int L, const float (&sh_rem)[kMaxTrkTaps], float2& ph, float2 (&acc)[kMaxTrkTaps + 1], bool probe, uint64_t& swait)
{
    const ChunkNco q = chunk_nco(p);
    constexpr int isz = item_bytes<IT>();
    const uint64_t nbytes = iq_items * (uint64_t)isz;
    const uintptr_t s0 = reinterpret_cast<uintptr_t>(iq) + (uintptr_t)p.off * isz;  // byte address of sample 0
    uintptr_t bstart[2];
    if (!pf_ok)
        {
            // a prefetch into buffer 0 that missed this call may still be landing, its
            // rows from other waves than this fetch's: let it land before refilling
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    // a tail of at most kTrkThreads samples rides with the last whole chunk (the
    // buffers hold chunk + kTrkThreads items): no loop iteration of its own
    int nch = (vl + chunk - 1) / chunk;
    if (nch > 1 && vl - (nch - 1) * chunk <= kTrkThreads) --nch;
    auto len = [&](int j) { return j == nch - 1 ? vl - j * chunk : chunk; };
    bstart[0] = pf_ok ? pf_start[0] : stream_fetch(iq, nbytes, p.off * isz, len(0) * isz, sb, 0);
    bstart[1] = 0;
    // chunk 1 came with chunk 0 (into the other buffer) when the prefetch covered it
    const bool pf1 = pf_ok && pf_start[1] != 0 && nch > 1;
    if (pf1) bstart[1] = pf_start[1];
    for (int j = 0; j < nch; ++j)
        {
            // a workgroup barrier waits only on lgkmcnt and LDS DMA is tracked per
            // wave in vmcnt: every issuing wave drains its own DMA (chunk j, and for
            // j == 0 the prefetch waves 1.. issued during the previous loop update)
            // before the barrier hands the buffer to the other waves
            const uint64_t w0 = probe ? wall_clock64() : 0;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (probe) swait += wall_clock64() - w0;
            if (j + 1 < nch && !(j == 0 && pf1))
                bstart[(j + 1) & 1] =
                    stream_fetch(iq, nbytes, (p.off + (int64_t)(j + 1) * chunk) * isz, len(j + 1) * isz, sb + ((j + 1) & 1) * sbuf_bytes, 0);
            const char* buf = sb + (j & 1) * sbuf_bytes;
            const int boff = (int)((int64_t)s0 - (int64_t)bstart[j & 1]);
            const int nend = j * chunk + len(j);
            for (int n0 = j * chunk; n0 < nend;)
                {
                    // E/P/L calls: two kWinCore blocks as one chunk of 2 kSpl samples per lane
                    // where they are whole and need no wrap -- twice the gathers in flight per
                    // wait (the lane's samples and their order are those of the two blocks;
                    // five taps or the data tap at this width spill)
                    if (KT == 3 && !DATA && n0 + 2 * kWinCore <= nend && q.wrap == 2)
                        {
                            correlate_chunk<IT, 2, 2, true, KT, DATA, 2 * kSpl>(iq, nullptr, s_code, s_data, p, q, n0, vl, L,
                                sh_rem, ph, acc, buf, boff);
                            n0 += 2 * kWinCore;
                        }
                    else
                        {
                            correlate_chunk_any<IT, 2, KT, DATA>(iq, nullptr, s_code, s_data, p, q, n0, vl, L, sh_rem, ph, acc,
                                buf, boff);
                            n0 += kWinCore;
                        }
                }
        }
}

// One call's NCO and read plan from the loop state (lane-uniform): computed by
// wave 0 at the end of the previous call's update, where the state is still in
// registers (launch start: by lane 0 from the LDS copy).
__device__ __forceinline__ Prep make_prep(const TrkConst& c, const TrkHot& t, bool go_epoch, uint64_t iq_first,
    uint64_t iq_items, int vl, int K, int L, bool use_window, bool streamed, int stream_chunk, int64_t win_base,
    int64_t pf_first)
{
    Prep p{};
    const int64_t off = (int64_t)(t.next_sample - iq_first);
    p.go = go_epoch && t.state >= 2 && t.state <= 4 && t.next_sample >= iq_first &&
           (uint64_t)off + (uint64_t)vl <= iq_items;
    p.off = off;
    p.narrow = t.narrow;
    p.woff = -1;
    if (use_window && win_base != INT64_MIN && off >= win_base && off - win_base + vl <= kWinCore + kHalo)
        p.woff = (int32_t)(off - win_base);
    p.pf_ok = streamed && pf_first != INT64_MIN && off >= pf_first &&
              off + min(vl, stream_chunk) <= pf_first + stream_chunk + kHalo;
    if (p.go)
        {
            // do_correlation_step's float arguments (:1069-1075); the
            // reference's phasors (cos r, -sin r) and exp(-j step)
            // (cpu_multicorrelator_real_codes.cc:114-123) as angles
            const float rem_carr = t.rem_carr_phase_rad;
            const float carr_step = (float)t.carrier_phase_step_rad;
            p.rem_code = (float)t.rem_code_phase_chips * (float)c.code_samples_per_chip;
            p.code_step = (float)t.code_phase_step_chips * (float)c.code_samples_per_chip;
            p.psi0 = -(double)rem_carr;
            p.theta = -(double)carr_step;
            // index range of the call (monotone in n for step > 0)
            // static tap indices throughout: a run-time index into p
            // (hdshift) sent the whole Prep through scratch
            float smin = 1e30f, smax = -1e30f;
#pragma unroll
            for (int k = 0; k < kMaxTrkTaps; ++k)
                {
                    if (k < K)
                        {
                            const float sr =
                                gsdr::sub_rn(t.narrow ? c.shifts_narrow[k] : c.shifts[k], p.rem_code);
                            smin = fminf(smin, sr);
                            smax = fmaxf(smax, sr);
                        }
                }
            const float lo = floorf(smin);
            const float hi = floorf(gsdr::add_rn(gsdr::mul_rn(p.code_step, (float)(vl - 1)), smax));
            const float Lf = (float)L;
            const bool mono = p.code_step >= 0.0f;
            p.wrap = (mono && lo >= -(float)kCodeMargin && hi < Lf + (float)kCodeMargin)
                         ? 2
                         : ((mono && lo >= -Lf && hi < 2.0f * Lf) ? 1 : 0);
            if (c.high_dyn)
                {
                    p.hd = 1;
                    p.theta_rate = -(double)(float)t.carrier_phase_rate_step_rad;
                    p.code_rate = (float)t.code_phase_rate_step_chips * (float)c.code_samples_per_chip;
                    unsigned int shs = 0;
                    p.hdshift[0] = 0;
#pragma unroll
                    for (int k = 1; k < kMaxTrkTaps; ++k)
                        {
                            if (k < K)
                                {
                                    const float* sk = t.narrow ? c.shifts_narrow : c.shifts;
                                    shs += (int)roundf((sk[k] - sk[k - 1]) / p.code_step);
                                    p.hdshift[k] = (int)shs;
                                }
                        }
                }
            const double w = p.theta * (double)kTrkThreads;
            float sn, cs;
            sincosf((float)fma(-rint(w * 0.15915494309189533576888376337251), 6.283185307179586476925286766559, w),
                &sn, &cs);
            p.wstep = make_float2(cs, sn);
        }
    return p;
}

// grid = channels; one kTrkThreads-lane workgroup per channel.  Wave 0 holds the
// mutable loop state in registers for the whole launch (uniform across its
// lanes); the configuration comes through scalar loads; the histories indexed at
// run time (CN0 buffer, DLL filter), the replica and the next call's input window
// sit in LDS.  While wave 0 runs the loop update of call e, every lane fetches
// the samples call e+1 will most likely read (the consumed count is one code
// period +-1 sample), so the update hides the HBM latency.
template <int IT>
__global__ void __launch_bounds__(kTrkThreads) trk_kernel(const TrkConst* __restrict__ consts,
    TrkChan* __restrict__ chans, const float* const* __restrict__ codes, const float* const* __restrict__ data_codes,
    const void* __restrict__ iq, uint64_t iq_first, uint64_t iq_items, uint32_t max_epochs, gsdr_trk_epoch* __restrict__ out,
    uint32_t* __restrict__ nout, int code_pad, int data_pad, uint64_t* __restrict__ timing, int timing_wall, int stream_chunk,
    int sbuf_bytes)
{
    // LDS: [replica | data replica (pilot tracking) | next call's input window]
    extern __shared__ float s_dyn[];
    // replicas with kCodeMargin wrapped samples on each side: s_code[-M .. L+M)
    float* s_code = s_dyn + kCodeMargin;
    float* s_data = s_dyn + code_pad + kCodeMargin;
    float2* s_win = reinterpret_cast<float2*>(s_dyn + code_pad + data_pad);
    char* s_sb = reinterpret_cast<char*>(s_dyn + code_pad + data_pad);  // streamed calls: two chunk buffers
    __shared__ LoopFilter s_lfs[2];  // code loop filter: current slot and wave 3's speculative one
    __shared__ int s_lfi;
    __shared__ DllPllSpec s_spec;
    __shared__ int s_spec_e;
    __shared__ DllSpec s_dspec;
    __shared__ int s_dspec_e;
    __shared__ float2 s_pbuf[kMaxCn0];
    __shared__ __attribute__((aligned(16))) float s_cn[3][kMaxCn0];  // cn0_and_lock's per-element terms
    __shared__ __attribute__((aligned(16))) float s_evm_buf[2 * kMaxCn0];  // evm_of's (wave 1)
    __shared__ double s_evm;
    __shared__ int s_evm_e;
    __shared__ Cn0Spec s_cn0;  // wave 2's lock test of the call (cn0_and_lock)
    __shared__ int s_cn0_e;
    __shared__ PlanIn s_plan;  // wave 0's loop state for wave 1's next-call plan
    __shared__ uint64_t s_w2t[3];  // GSDR_TRK_TIMING: wave 2's lock test start / end, wave 1's EVM end
    __shared__ int s_plan_e, s_prep_e;
    __shared__ int s_state;
    __shared__ Prep prep;
    __shared__ float2 s_red[kTrkThreads / 64][kMaxTrkTaps + 1];
    // the loop state lives in LDS between calls and in wave 0's registers only
    // during the loop update, so the correlation keeps its registers for loads
    // in flight (with the state resident for the whole launch the kernel sat at
    // 256 VGPRs and the compiler serialised the sample loads)
    __shared__ TrkHot s_t;
    __shared__ int s_overrun;  // the channel fell behind the input (one loss-of-lock record)
    const int ch = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const TrkConst& c = consts[ch];
    TrkChan* gc = chans + ch;
    // The tracking loop is a latency chain that shares its CUs with the
    // acquisition grid running on another queue: raise the issue priority.
    __builtin_amdgcn_s_setprio(3);
    if (tid == 0)
        {
            s_t = gc->h;
            s_lfs[0] = gc->code_filter;
            s_lfi = 0;
            s_spec_e = -1;
            s_dspec_e = -1;
            s_evm_e = -1;
            s_cn0_e = -1;
            s_plan_e = -1;
            s_prep_e = -1;
            s_state = s_t.state;
            s_overrun = 0;
        }
    if (tid < kMaxCn0) s_pbuf[tid] = gc->prompt_buffer[tid];
    __syncthreads();
    if (s_state < 2 || s_state > 4)
        {
            if (tid == 0) nout[ch] = 0;
            return;
        }
    const int K = c.n_taps;
    const int L = c.code_samples;
    const int vl = c.vector_length;
    // calls of at most kWinCore samples: the next call's window staged by waves 3.. through
    // registers (the streamed path's LDS-DMA prefetch for them measured 181 -> 213 ticks of
    // correlation per C2 call, profiles/r06r)
    const bool use_window = vl <= kWinCore;
    const bool streamed = !use_window && stream_chunk > 0;
    const bool data = c.track_pilot != 0;
    {
        const float* cd = codes[ch];
        for (int i = tid - kCodeMargin; i < L + kCodeMargin; i += kTrkThreads) s_code[i] = cd[((i % L) + L) % L];
        if (data)
            {
                const float* dd = data_codes[ch];
                for (int i = tid - kCodeMargin; i < L + kCodeMargin; i += kTrkThreads) s_data[i] = dd[((i % L) + L) % L];
            }
    }
    int64_t win_base = INT64_MIN;  // absolute-index base of the staged window (uniform)
    int lfi0 = 0;                  // wave 0: the current code loop filter slot (s_lfi)
    int64_t pf_first = INT64_MIN;  // streamed calls: first sample of the prefetched chunk 0 (uniform)
    uintptr_t pf_start[2] = {0, 0};  // and the byte addresses chunks 0 / 1's LDS buffers start at (0: not fetched)
    uint32_t e = 0;
    for (;; ++e)
        {
            uint64_t tm0 = 0, tm1 = 0, tm2 = 0, swait = 0;
            if (timing && tid == 0) tm0 = wall_clock64();
            if (tid == 0 && e == 0)
                {
                    const TrkHot& t = s_t;
                    if (e == 0 && t.state >= 2 && t.state <= 4 && t.next_sample < iq_first && max_epochs > 0)
                        {
                            // the channel's next call starts before the oldest item the
                            // caller provides (a ring that moved past a stalled channel):
                            // it can never continue, so report it as a loss of lock
                            // (event 3, the Channel FSM re-acquires) instead of stalling
                            gsdr_trk_epoch r{};
                            r.sample_counter = t.next_sample;
                            r.state = t.state;
                            r.flags = GSDR_TRK_F_LOSS_OF_LOCK | GSDR_TRK_F_OVERRUN;
                            r.carrier_doppler_hz = t.carrier_doppler_hz;
                            r.code_freq_chips = t.code_freq_chips;
                            r.cn0_db_hz = t.cn0_db_hz;
                            out[(size_t)ch * max_epochs] = r;
                            clear_tracking_vars(s_t);
                            s_t.state = 0;
                            s_overrun = 1;
                        }
                    prep = make_prep(c, t, e < max_epochs, iq_first, iq_items, vl, K, L, use_window, streamed,
                        stream_chunk, win_base, pf_first);
                }
            __syncthreads();
            if (!prep.go) break;
            if (timing && tid == 0) tm1 = wall_clock64();
            // ---- correlation: lane-interleaved samples, fp64 phasor anchor + fp32 steps
            // the plan read from LDS where it is used (a register copy lived across the
            // whole correlation and the allocator spilled it); the offset is read once,
            // before wave 0 can write the next plan
            const Prep& p = prep;
            const int64_t p_off = p.off;
            float2 acc[kMaxTrkTaps + 1];
#pragma unroll
            for (int k = 0; k <= kMaxTrkTaps; ++k) acc[k] = make_float2(0.f, 0.f);
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
            for (int k = 0; k < kMaxTrkTaps; ++k)
                sh_rem[k] = gsdr::sub_rn(p.narrow ? c.shifts_narrow[k] : c.shifts[k], p.rem_code);
            if (p.hd)
                {
                    const float* sk = p.narrow ? c.shifts_narrow : c.shifts;
                    correlate_call_hd<IT>(iq, s_win, s_code, s_data, p, vl, L, K, data, sk[0], sk[c.iP], acc);
                }
            else if (streamed)
                {
                    const bool sw = timing && tid == 0;
                    if (K <= 3)
                        correlate_call_stream<IT, 3, false>(iq, iq_items, s_sb, sbuf_bytes, stream_chunk, p.pf_ok, pf_start,
                            s_code, s_data, p, vl, L, sh_rem, ph, acc, sw, swait);
                    else if (!data)
                        correlate_call_stream<IT, kMaxTrkTaps, false>(iq, iq_items, s_sb, sbuf_bytes, stream_chunk, p.pf_ok,
                            pf_start, s_code, s_data, p, vl, L, sh_rem, ph, acc, sw, swait);
                    else
                        correlate_call_stream<IT, kMaxTrkTaps, true>(iq, iq_items, s_sb, sbuf_bytes, stream_chunk, p.pf_ok,
                            pf_start, s_code, s_data, p, vl, L, sh_rem, ph, acc, sw, swait);
                }
            else if (K <= 3)
                correlate_call<IT, 3, false>(iq, s_win, s_code, s_data, p, vl, L, sh_rem, ph, acc);
            else if (!data)
                correlate_call<IT, kMaxTrkTaps, false>(iq, s_win, s_code, s_data, p, vl, L, sh_rem, ph, acc);
            else
                correlate_call<IT, kMaxTrkTaps, true>(iq, s_win, s_code, s_data, p, vl, L, sh_rem, ph, acc);
#pragma unroll
            for (int k = 0; k <= kMaxTrkTaps; ++k)
                {
                    if (k < K || (k == kMaxTrkTaps && data))
                        {
                            // wave sums by DPP (the total in lane 63)
                            acc[k].x = gsdr::wave_sum_lane63(acc[k].x);
                            acc[k].y = gsdr::wave_sum_lane63(acc[k].y);
                        }
                }
            if (lane == 63)
                {
#pragma unroll
                    for (int k = 0; k <= kMaxTrkTaps; ++k) s_red[wave][k] = acc[k];
                }
            __syncthreads();  // partials visible; every read of the LDS window done
            if (timing && tid == 0) tm2 = wall_clock64();
            // lane k sums tap k over the waves in wave order (one batch of LDS reads
            // instead of a serial read per partial), then every lane takes the totals
            // by readlane; E/P/L are the same sums
            auto tap_totals = [&](float2 (&taps)[kMaxTrkTaps + 1], float2 (&epl)[3]) {
                float2 mine = make_float2(0.f, 0.f);
                if (lane <= kMaxTrkTaps)
                    {
                        float2 v[kTrkThreads / 64];
#pragma unroll
                        for (int w = 0; w < kTrkThreads / 64; ++w) v[w] = s_red[w][lane];
#pragma unroll
                        for (int w = 0; w < kTrkThreads / 64; ++w)
                            {
                                mine.x += v[w].x;
                                mine.y += v[w].y;
                            }
                    }
#pragma unroll
                for (int k = 0; k <= kMaxTrkTaps; ++k)
                    taps[k] = (k < K || (k == kMaxTrkTaps && data)) ? make_float2(lane_f(mine.x, k), lane_f(mine.y, k))
                                                                   : make_float2(0.f, 0.f);
                const int ix[3] = {c.iE, c.iP, c.iL};
#pragma unroll
                for (int q = 0; q < 3; ++q) epl[q] = make_float2(lane_f(mine.x, ix[q]), lane_f(mine.y, ix[q]));
            };
            if (wave == 3)
                {
                    // this call's code loop (DLL discriminator and filter) on a copy of
                    // the state, into the code loop filter slot that is not current; wave
                    // 1 runs the carrier loop at the same time (take_dll_pll joins them).
                    // Before this wave's share of the window staging / prefetch, which
                    // only has to land before the next call
                    TrkHot t3 = s_t;
                    if (t3.state == 2 || t3.state == 4)
                        {
                            float2 taps[kMaxTrkTaps + 1], epl[3];
                            tap_totals(taps, epl);
                            if (t3.state == 2)
                                {
                                    if (c.veml)
                                        {
                                            t3.VE_accu = taps[0];
                                            t3.VL_accu = taps[4];
                                        }
                                    t3.E_accu = epl[0];
                                    t3.P_accu = epl[1];
                                    t3.L_accu = epl[2];
                                    t3.spc = c.early_late_space_chips;
                                }
                            else
                                save_correlation_results(c, t3, taps, epl);
                            // the filter in registers, written to the other slot after
                            const int cur = s_lfi;
                            LfReg lf3 = lf_load(s_lfs[cur]);
                            const double base = run_dll(c, t3, lf3);
                            if (lane == 0)
                                {
                                    LoopFilter& d = s_lfs[cur ^ 1];
                                    d = s_lfs[cur];
                                    d.inputs[0] = lf3.i0;
                                    d.inputs[1] = lf3.i1;
                                    d.inputs[2] = lf3.i2;
                                    d.inputs[3] = lf3.i3;
                                    d.outputs[0] = lf3.o0;
                                    d.outputs[1] = lf3.o1;
                                    d.outputs[2] = lf3.o2;
                                    d.outputs[3] = lf3.o3;
                                    d.idx = lf3.idx;
                                    DllSpec r;
                                    r.code_freq_base = base;
                                    r.log_err2 = t3.log_err[2];
                                    r.log_err3 = t3.log_err[3];
                                    s_dspec = r;
                                    __hip_atomic_store(&s_dspec_e, (int)e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                        }
                }
            // ---- stage the window the next call most likely reads, [off + vl - kHalo/2,
            // +kWinCore+kHalo), into LDS: waves 3.. only (wave 3 after its code loop),
            // while wave 0 runs the loop update, wave 1 the carrier loop and the EVM and
            // wave 2 the lock test (every read of the current window is done), so wave 0
            // issues no global loads that a vmcnt wait inside its update would wait for
            const int64_t nb = p_off + vl - kHalo / 2;
            if (use_window && wave >= 3)
                {
                    // two batches of loads in flight (the update hides their latency)
                    constexpr int kW = kTrkThreads - 192;
                    constexpr int kIt = (kWinCore + kHalo + kW - 1) / kW;
                    constexpr int kB = (kIt + 1) / 2;
                    // one 64-bit base per call and constant steps (per-item 64-bit
                    // offsets were hoisted out of the call loop and held 26 VGPRs)
                    const int i0 = tid - 192;
                    const int64_t g0 = nb + i0;
#pragma unroll
                    for (int j0 = 0; j0 < kIt; j0 += kB)
                        {
                            float2 wv[kB];
#pragma unroll
                            for (int j = 0; j < kB; ++j)
                                {
                                    const int64_t g = g0 + (int64_t)((j0 + j) * kW);
                                    wv[j] = (j0 + j < kIt && i0 + (j0 + j) * kW < kWinCore + kHalo && (uint64_t)g < iq_items)
                                                ? load_iq<IT>(iq, g)
                                                : make_float2(0.f, 0.f);
                                }
#pragma unroll
                            for (int j = 0; j < kB; ++j)
                                {
                                    const int i = i0 + (j0 + j) * kW;
                                    if (j0 + j < kIt && i < kWinCore + kHalo) s_win[i] = wv[j];
                                }
                        }
                }
            if (streamed)
                {
                    // chunks 0 and 1 of the call most likely next, into the two buffers,
                    // fetched by waves 3.. while wave 0 runs the loop update (its own
                    // memory waits stay unaffected) and waves 1 / 2 the speculative
                    // DLL/PLL and the EVM: the call's first in-call fetch is then chunk 2,
                    // issued a whole chunk of correlation ahead
                    const int64_t nb = p_off + vl - kHalo / 2;
                    const uint64_t nbytes = iq_items * (uint64_t)item_bytes<IT>();
                    // sized for the tail a last chunk may carry whatever this call's split
                    // (the buffers hold chunk + kTrkThreads + kHalo items): a call
                    // correlates the channel's constant vector_length samples
                    // (do_correlation_step, :1064-1076), so the split cannot change between
                    // calls today, but the prefetch no longer depends on that
                    const int pfn = (stream_chunk + kTrkThreads + kHalo) * item_bytes<IT>();
                    pf_start[0] = stream_fetch(iq, nbytes, nb * item_bytes<IT>(), pfn, s_sb, 3);
                    pf_start[1] = vl > stream_chunk + kTrkThreads
                                      ? stream_fetch(iq, nbytes, (nb + stream_chunk) * item_bytes<IT>(), pfn, s_sb + sbuf_bytes, 3)
                                      : 0;
                    pf_first = nb;
                }
            if (wave == 1)
                {
                    // this call's DLL/PLL on a copy of the state, into the code loop
                    // filter slot that is not current (take_dll_pll)
                    TrkHot t1 = s_t;
                    if (t1.state == 2 || t1.state == 4)
                        {
                            float2 taps[kMaxTrkTaps + 1], epl[3];
                            tap_totals(taps, epl);
                            const uint64_t n_read = t1.next_sample;
                            if (t1.pull_in_transitory &&
                                (n_read < c.acq_sample_stamp || n_read - c.acq_sample_stamp >= c.pull_in_span))
                                t1.pull_in_transitory = 0;
                            if (t1.state == 2)
                                {
                                    if (c.veml)
                                        {
                                            t1.VE_accu = taps[0];
                                            t1.VL_accu = taps[4];
                                        }
                                    t1.E_accu = epl[0];
                                    t1.P_accu = epl[1];
                                    t1.L_accu = epl[2];
                                    t1.spc = c.early_late_space_chips;
                                }
                            else
                                save_correlation_results(c, t1, taps, epl);
                            run_pll(c, t1);
                            if (lane == 0)
                                {
                                    DllPllSpec r;
                                    r.carrier_doppler_hz = t1.carrier_doppler_hz;
                                    r.P_accu_old = t1.P_accu_old;
                                    r.cf_w = t1.cf_w;
                                    r.cf_x = t1.cf_x;
                                    r.log_err[0] = t1.log_err[0];
                                    r.log_err[1] = t1.log_err[1];
                                    s_spec = r;
                                    __hip_atomic_store(&s_spec_e, (int)e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                            // then the EVM (an output only) with a full prompt buffer, which
                            // wave 0 takes for the record when the call stays locked: the
                            // buffer's other elements and this call's prompt (wave 2 writes
                            // only this call's element)
                            if (t1.cn0_estimation_counter >= c.cn0_samples)
                                {
                                    const double evm = evm_of(c, t1.cn0_estimation_counter, t1.P_accu, s_pbuf, s_evm_buf, lane);
                                    if (lane == 0)
                                        {
                                            if (timing) s_w2t[2] = wall_clock64();
                                            s_evm = evm;
                                            __hip_atomic_store(&s_evm_e, (int)e, __ATOMIC_RELEASE,
                                                __HIP_MEMORY_SCOPE_WORKGROUP);
                                        }
                                }
                            // then the next call's plan from wave 0's state after its
                            // locked branch (wave 0 overrides it on a loss of lock)
                            while (__hip_atomic_load(&s_plan_e, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)e)
                                __builtin_amdgcn_s_sleep(1);
                            const PlanIn q = s_plan;
                            t1.carrier_phase_step_rad = q.carrier_phase_step_rad;
                            t1.carrier_phase_rate_step_rad = q.carrier_phase_rate_step_rad;
                            t1.rem_code_phase_chips = q.rem_code_phase_chips;
                            t1.code_phase_step_chips = q.code_phase_step_chips;
                            t1.code_phase_rate_step_chips = q.code_phase_rate_step_chips;
                            t1.next_sample = q.next_sample;
                            t1.rem_carr_phase_rad = q.rem_carr_phase_rad;
                            t1.state = q.state;
                            t1.narrow = q.narrow;
                            const Prep pn = make_prep(c, t1, e + 1 < max_epochs, iq_first, iq_items, vl, K, L, use_window,
                                streamed, stream_chunk, use_window ? nb : win_base, streamed ? nb : pf_first);
                            if (lane == 0)
                                {
                                    prep = pn;
                                    __hip_atomic_store(&s_prep_e, (int)e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                        }
                }
            if (wave == 2)
                {
                    // this call's lock test (CN0 estimate, lock detector, the prompt
                    // buffer) on a copy of the state, which wave 0 takes after its locked
                    // branch
                    TrkHot t2 = s_t;
                    if (t2.state == 2 || t2.state == 4)
                        {
                            float2 taps[kMaxTrkTaps + 1], epl[3];
                            tap_totals(taps, epl);
                            const uint64_t n_read = t2.next_sample;
                            if (t2.pull_in_transitory &&
                                (n_read < c.acq_sample_stamp || n_read - c.acq_sample_stamp >= c.pull_in_span))
                                {
                                    t2.pull_in_transitory = 0;
                                    t2.carrier_lock_fail_counter = 0;
                                    t2.code_lock_fail_counter = 0;
                                }
                            const double coh =
                                t2.state == 2 ? c.code_period : c.code_period * (double)c.extend_correlation_symbols;
                            pre_lock(c, t2, taps, epl, n_read);
                            if (timing && lane == 0) s_w2t[0] = wall_clock64();
                            const int locked = cn0_and_lock(c, t2, s_pbuf, s_cn, coh, lane);
                            if (lane == 0)
                                {
                                    if (timing) s_w2t[1] = wall_clock64();
                                    cn0_publish(s_cn0, t2, locked);
                                    __hip_atomic_store(&s_cn0_e, (int)e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                        }
                }
            if (wave == 0)
                {
                    TrkHot t = s_t;
                    uint64_t tmA = 0;
                    if (timing) tmA = wall_clock64();
                    float2 taps[kMaxTrkTaps + 1], epl[3];
                    tap_totals(taps, epl);
                    const uint64_t n_read = t.next_sample;
                    const int32_t state0 = t.state;
                    // pull-in transitory check at the top of general_work (:1794-1803):
                    // pull_in_time_s < (nitems_read - stamp) / (int)fs_in, integer division
                    if (t.pull_in_transitory &&
                        (n_read < c.acq_sample_stamp || n_read - c.acq_sample_stamp >= c.pull_in_span))
                        {
                            t.pull_in_transitory = 0;
                            t.carrier_lock_fail_counter = 0;
                            t.code_lock_fail_counter = 0;
                        }
                    EpochOut o;
                    uint64_t pr[3] = {0, 0, 0};
                    uint64_t tm3 = 0;
                    if (timing) tm3 = wall_clock64();
                    SpecLink sl{&s_spec, &s_dspec, &s_dspec_e, &s_spec_e, s_lfs, &s_lfi, lfi0, (int)e};
                    after_correlation(c, t, gc, sl, taps, epl, n_read, o, timing != nullptr, pr);
                    t.next_sample = n_read + (uint64_t)(int64_t)t.current_prn_length_samples;
                    // the next call's plan (the window / chunk-0 prefetch of this iteration
                    // starts at nb): states 2 / 4 on wave 1 from the state published here,
                    // before the lock test's results (they change the plan only on a loss
                    // of lock: state 0, no call); state 3 here
                    const bool plan_w1 = state0 == 2 || state0 == 4;
                    Prep pn{};
                    if (plan_w1)
                        {
                            if (lane == 0)
                                {
                                    PlanIn q;
                                    q.carrier_phase_step_rad = t.carrier_phase_step_rad;
                                    q.carrier_phase_rate_step_rad = t.carrier_phase_rate_step_rad;
                                    q.rem_code_phase_chips = t.rem_code_phase_chips;
                                    q.code_phase_step_chips = t.code_phase_step_chips;
                                    q.code_phase_rate_step_chips = t.code_phase_rate_step_chips;
                                    q.next_sample = t.next_sample;
                                    q.rem_carr_phase_rad = t.rem_carr_phase_rad;
                                    q.state = t.state;
                                    q.narrow = t.narrow;
                                    s_plan = q;
                                    __hip_atomic_store(&s_plan_e, (int)e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                                }
                        }
                    else
                        pn = make_prep(c, t, e + 1 < max_epochs, iq_first, iq_items, vl, K, L, use_window, streamed,
                            stream_chunk, use_window ? nb : win_base, streamed ? nb : pf_first);
                    bool lost = false;
                    uint64_t tjoin = 0;
                    if (state0 == 2 || state0 == 4)
                        {
                            if (timing) tjoin = wall_clock64();
                            while (__hip_atomic_load(&s_cn0_e, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)e)
                                __builtin_amdgcn_s_sleep(1);
                            const Cn0Spec r = s_cn0;
                            if (r.locked)
                                {
                                    cn0_apply(t, r);
                                    o.evm = r.locked == 2;
                                }
                            else
                                {
                                    // loss of lock: cn0_and_tracking_lock_status returned
                                    // false and the reference's call ends there (:1828-1845,
                                    // :2032-2040), so the locked branch above is void: the
                                    // call is rebuilt from its start state
                                    t = s_t;
                                    if (t.pull_in_transitory &&
                                        (n_read < c.acq_sample_stamp || n_read - c.acq_sample_stamp >= c.pull_in_span))
                                        t.pull_in_transitory = 0;
                                    pre_lock(c, t, taps, epl, n_read);
                                    cn0_apply(t, r);
                                    clear_tracking_vars(t);
                                    if (c.track_pilot) t.P_data_accu = make_float2(0.f, 0.f);
                                    t.state = 0;
                                    init_out(o);
                                    o.flags = GSDR_TRK_F_LOSS_OF_LOCK | (t.flag_pll_180 ? GSDR_TRK_F_PLL_180 : 0);
                                    sl.lfi = lfi0;  // the DLL/PLL results were not taken
                                    t.next_sample = n_read + (uint64_t)(int64_t)t.current_prn_length_samples;
                                    lost = true;
                                }
                        }
                    if (sl.lfi != lfi0)
                        {
                            lfi0 = sl.lfi;
                            if (lane == 0) s_lfi = lfi0;
                        }
                    uint64_t tevm0 = 0, tevm1 = 0;
                    if (o.evm)
                        {
                            if (timing) tevm0 = wall_clock64();
                            while (__hip_atomic_load(&s_evm_e, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)e)
                                __builtin_amdgcn_s_sleep(1);
                            t.evm = s_evm;
                            if (timing) tevm1 = wall_clock64();
                        }
                    if (lane == 0)
                        {
                            gsdr_trk_epoch r;
                            r.sample_counter = n_read;
                            r.state = state0;
                            r.consumed = t.current_prn_length_samples;
#pragma unroll
                            for (int k = 0; k < 5; ++k)
                                {
                                    r.taps[2 * k] = taps[k].x;
                                    r.taps[2 * k + 1] = taps[k].y;
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
                            r.data_prompt[0] = data ? taps[kMaxTrkTaps].x : 0.0F;
                            r.data_prompt[1] = data ? taps[kMaxTrkTaps].y : 0.0F;
                            r.carrier_rate = (float)t.carrier_phase_rate_step_rad;
                            r.code_rate = (float)t.code_phase_rate_step_chips;
#pragma unroll
                            for (int i = 0; i < 5; ++i) r.log_accu[i] = o.log_accu[i];
                            r.carr_phase_error_hz = t.log_err[0];
                            r.carr_error_filt_hz = t.log_err[1];
                            r.code_error_chips = t.log_err[2];
                            r.code_error_filt_chips = t.log_err[3];
                            r.reserved = 0;
                            out[(size_t)ch * max_epochs + e] = r;
                            if (timing)
                                {
                                    uint64_t* tr = timing + ((size_t)ch * max_epochs + e) * kTimingSlots;
                                    tr[0] = tm0;
                                    tr[1] = tm1;
                                    tr[2] = tm2;
                                    tr[3] = tmA;
                                    tr[4] = tm3;
                                    tr[5] = pr[0] ? pr[0] : tm3;
                                    tr[6] = pr[1] ? pr[1] : tr[5];
                                    tr[7] = pr[2] ? pr[2] : tr[6];
                                    tr[8] = wall_clock64();
                                    tr[10] = swait;
                                    const bool w2 = tjoin != 0;
                                    tr[11] = w2 && s_w2t[0] >= tm2 ? s_w2t[0] - tm2 : 0;
                                    tr[12] = w2 && s_w2t[1] >= tm2 ? s_w2t[1] - tm2 : 0;
                                    tr[13] = w2 && tjoin >= tm2 ? tjoin - tm2 : 0;
                                    tr[14] = tevm0 && s_w2t[2] >= tm2 ? s_w2t[2] - tm2 : 0;
                                    tr[15] = tevm0 >= tm2 && tevm0 ? tevm0 - tm2 : 0;
                                    tr[16] = tevm1 >= tm2 && tevm1 ? tevm1 - tm2 : 0;
                                }
                        }
                    if (lane == 0) s_t = t;
                    if (!plan_w1)
                        {
                            if (lane == 0) prep = pn;
                        }
                    else if (lost)
                        {
                            // no next call: after wave 1's plan, so this write lands last
                            while (__hip_atomic_load(&s_prep_e, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) != (int)e)
                                __builtin_amdgcn_s_sleep(1);
                            if (lane == 0) prep.go = 0;
                        }
                    if (timing && lane == 0) timing[((size_t)ch * max_epochs + e) * kTimingSlots + 9] = wall_clock64();
                }
            if (use_window) win_base = nb;
            // the next iteration's prep barrier orders the window writes and s_red reuse
        }
    __syncthreads();
    if (tid == 0)
        {
            gc->h = s_t;
            gc->code_filter = s_lfs[s_lfi];
            nout[ch] = e + (uint32_t)s_overrun;
        }
    if (tid < kMaxCn0) gc->prompt_buffer[tid] = s_pbuf[tid];
}

// A secondary code / preamble string as the register acquire_secondary compares
// with: the register holds the signs of the last pushes (1 = real < 0), newest at
// bit 0, so string index i (oldest first) sits at bit len-1-i; a match for
// real < 0 is character '0' (:923-967), so the register bit is 1 where the
// character is '0'.  str_bits: bit i = (string[i] == '1').
void code_registers(const char* str, int len, uint32_t reg[5], uint32_t str_bits[5])
{
    for (int w = 0; w < 5; ++w) reg[w] = str_bits[w] = 0u;
    for (int i = 0; i < len; ++i)
        {
            const int bit = len - 1 - i;
            if (str[i] == '0') reg[bit >> 5] |= 1u << (bit & 31);
            if (str[i] == '1') str_bits[i >> 5] |= 1u << (i & 31);
        }
}

void set_secondary(TrkConst& c, const char* str, int len)
{
    c.sec_len = len;
    code_registers(str, len, c.preamble, c.sec_str);
}

}  // namespace

struct gsdr_trk
{
    int device{0};
    gsdr_trk_conf conf{};
    hipStream_t stream{nullptr};
    std::vector<TrkConst> h_consts;
    std::vector<TrkChan> h_chans;
    TrkConst* d_consts{nullptr};
    TrkChan* d_chans{nullptr};
    TrkChan* d_snap[2]{nullptr, nullptr};
    std::vector<float*> code_bufs;
    float** d_codes{nullptr};
    std::vector<float*> data_code_bufs;  // pilot tracking: data-component replicas
    float** d_data_codes{nullptr};
    std::vector<int> data_code_len;
    gsdr_trk_epoch* d_out{nullptr};
    uint32_t* d_nout{nullptr};
    uint32_t out_cap{0};
    void* d_iq{nullptr};
    uint64_t iq_cap{0};
    size_t lds_bytes{0};
    int code_pad{1024 + 2 * kCodeMargin};  // floats reserved for the padded replica ahead of the LDS window
    int data_pad{0};     // floats reserved for the data replica (pilot tracking)
    // GSDR_TRK_TIMING=1: per-phase clock64 stamps of every call, summarised on destroy
    bool timing_on{false};
    int timing_wall{0};  // GSDR_TRK_TIMING=2: constant-rate wall clock instead of the shader clock
    uint64_t* d_timing{nullptr};
    size_t timing_cap{0};
    double tsum[kTimingSlots]{};
    uint32_t timing_epochs{0};
    uint32_t* timing_nout{nullptr};
    uint64_t tcount{0};
    bool profiling{false};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_recs;
    std::vector<hipEvent_t> prof_pool;
    // recorded after every launch on the stream it used: host read-modify-writes of
    // d_chans (start / stop / get_channel) wait for it, so a launch in flight on a
    // caller stream cannot write a stale channel back over them
    hipEvent_t last_launch{nullptr};
    // gsdr_trk_submit_stream / gsdr_trk_collect: device records of the submission,
    // their pinned host image and the event of its copy
    struct Submission
    {
        // the kernel writes the records straight into pinned host memory (zero-copy):
        // no copy-engine hop between one advance's kernel and the next on the stream
        gsdr_trk_epoch* h_out{nullptr};
        uint32_t* h_nout{nullptr};
        uint32_t cap{0};  // records per channel the buffers hold
        uint32_t epochs{0};
        hipEvent_t done{nullptr};
    };
    static constexpr int kSubmissions = 2;  // in flight at once (collected oldest first)
    Submission sub[kSubmissions];
    int sub_head{0};   // the oldest pending submission
    int sub_count{0};  // pending submissions
    std::mutex mu;
    // held for a whole gsdr_trk_submit_stream: the slot it picks stays its own while
    // mu is released for the launch (a second submitter waits; a collect in between
    // takes only committed submissions and leaves sub_head + sub_count unchanged)
    std::mutex submit_mu;
};

namespace
{

size_t trk_item_bytes(int it) { return it == GSDR_ITEM_CSHORT ? 4 : (it == GSDR_ITEM_IBYTE ? 2 : 8); }

// constructor (dll_pll_veml_tracking.cc:85-560) for one channel slot, GPS L1 C/A
// Tracking_FLL_PLL_filter::set_params (tracking_FLL_PLL_filter.cc:23-58)
void cf_set_params(CfConst& p, float fll_bw, float pll_bw, int order)
{
    p = CfConst{};
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

// Exponential_Smoother::set_alpha (exponential_smoother.cc:29-41)
void sm_set(SmConst& k, float alpha, float min_value, float offset, int samples)
{
    k.alpha = alpha;
    if (k.alpha < 0) k.alpha = 0;
    if (k.alpha > 1) k.alpha = 1;
    k.one_minus_alpha = 1.0F - k.alpha;
    k.min_value = min_value;
    k.offset = offset;
    k.samples_init = std::max(1, samples);
}

// tap shifts (:466-507 / :850-862), in replica samples; the narrow set of the
// extended correlator (:1963-1977)
void set_shifts(const gsdr_trk_conf& cf, TrkConst& c)
{
    const float spc = (float)c.code_samples_per_chip;
    if (c.veml)
        {
            c.shifts[0] = -cf.very_early_late_space_chips * spc;
            c.shifts[1] = -cf.early_late_space_chips * spc;
            c.shifts[2] = 0.0F;
            c.shifts[3] = cf.early_late_space_chips * spc;
            c.shifts[4] = cf.very_early_late_space_chips * spc;
            c.shifts_narrow[0] = -cf.very_early_late_space_narrow_chips * spc;
            c.shifts_narrow[1] = -cf.early_late_space_narrow_chips * spc;
            c.shifts_narrow[2] = 0.0F;
            c.shifts_narrow[3] = cf.early_late_space_narrow_chips * spc;
            c.shifts_narrow[4] = cf.very_early_late_space_narrow_chips * spc;
        }
    else
        {
            c.shifts[0] = -cf.early_late_space_chips * spc;
            c.shifts[1] = 0.0F;
            c.shifts[2] = cf.early_late_space_chips * spc;
            c.shifts_narrow[0] = -cf.early_late_space_narrow_chips * spc;
            c.shifts_narrow[1] = 0.0F;
            c.shifts_narrow[2] = cf.early_late_space_narrow_chips * spc;
        }
}

// signal table of the constructor (dll_pll_veml_tracking.cc:170-430)
struct SignalParams
{
    double carrier_hz, period_s, chip_rate;
    int length_chips, samples_per_chip, symbols_per_bit, veml;
};
SignalParams signal_params(int signal)
{
    if (signal == GSDR_SIGNAL_GAL_1B) return {kGalE1Hz, kGalE1Period, kGalE1Rate, kGalE1Length, 2, 1, 1};
    if (signal == GSDR_SIGNAL_BDS_B1) return {kBdsB1Hz, kBdsB1Period, kBdsB1Rate, kBdsB1Length, 1, 20, 0};
    return {kGpsL1Hz, kGpsCaPeriod, kGpsCaRate, kGpsCaLength, 1, kGpsCaSymbolsPerBit, 0};
}

// constructor (dll_pll_veml_tracking.cc:85-560) for one channel slot
void init_channel(const gsdr_trk_conf& cf, TrkConst& c, TrkChan& ch)
{
    std::memset(&c, 0, sizeof(c));
    std::memset(&ch, 0, sizeof(ch));
    const SignalParams sp = signal_params(cf.signal);
    c.fs_in = cf.fs_in;
    c.code_period = sp.period_s;
    c.code_chip_rate = sp.chip_rate;
    c.signal_carrier_freq = sp.carrier_hz;
    c.veml = sp.veml;
    c.iE = c.veml ? 1 : 0;
    c.iP = c.veml ? 2 : 1;
    c.iL = c.veml ? 3 : 2;
    if (cf.signal == GSDR_SIGNAL_GAL_1B)
        {
            c.track_pilot = cf.track_pilot ? 1 : 0;
            c.secondary = c.track_pilot;
            if (c.secondary) set_secondary(c, kGalE1cSecondary, 25);
        }
    else if (cf.signal == GSDR_SIGNAL_BDS_B1)
        {
            // D1 by default; gsdr_trk_start switches GEO PRNs to the D2 preamble
            c.secondary = 1;
            set_secondary(c, kBdsB1Nh, 20);
            uint32_t reg[5], bits[5];
            code_registers(kBdsB1Nh, 20, reg, bits);
            c.data_sec_len = 20;
            c.data_sec_str = bits[0];
        }
    else
        set_secondary(c, kGpsCaPreamble, kPreambleLen);
    c.carrier_lock_threshold = cf.carrier_lock_th;
    c.early_late_space_chips = cf.early_late_space_chips;
    c.vector_length = (int32_t)cf.vector_length;
    c.code_length_chips = sp.length_chips;
    c.code_samples_per_chip = sp.samples_per_chip;
    c.symbols_per_bit = sp.symbols_per_bit;
    c.cn0_samples = cf.cn0_samples;
    c.cn0_min = cf.cn0_min;
    c.max_code_lock_fail = cf.max_code_lock_fail;
    c.max_carrier_lock_fail = cf.max_carrier_lock_fail;
    const uint64_t fsi = (uint64_t)(int64_t)(int)cf.fs_in;
    c.pull_in_span = ((uint64_t)cf.pull_in_time_s + 1) * fsi;
    c.bit_sync_span = ((uint64_t)cf.bit_synchronization_time_limit_s + 1) * fsi;
    c.extend_correlation_symbols = cf.extend_correlation_symbols;
    c.enable_fll_pull_in = cf.enable_fll_pull_in;
    c.enable_fll_steady_state = cf.enable_fll_steady_state;
    c.carrier_aiding = cf.carrier_aiding;
    c.n_taps = c.veml ? 5 : 3;
    set_shifts(cf, c);
    cf_set_params(c.cf, cf.fll_bw_hz, cf.pll_bw_hz, cf.pll_filter_order);
    cf_set_params(c.cf_narrow, cf.fll_bw_hz, cf.pll_bw_narrow_hz, cf.pll_filter_order);
    c.early_late_space_narrow_chips = cf.early_late_space_narrow_chips;
    c.dll_bw_narrow_hz = cf.dll_bw_narrow_hz;
    c.enable_ext = cf.extend_correlation_symbols > 1 ? 1 : 0;
    c.high_dyn = cf.high_dyn ? 1 : 0;
    // dll_pll_conf.cc:118-123: smoother_length < 1 is set to 1
    c.smoother_length = cf.smoother_length < 1 ? 1 : (int32_t)cf.smoother_length;
    // Exponential_Smoother defaults (exponential_smoother.h:58-63) + dll_pll_veml_tracking.cc:540-552
    sm_set(c.sm[0], cf.cn0_smoother_alpha, 25.0F, 12.0F, cf.cn0_smoother_samples / (int)(c.code_period * 1000.0));
    sm_set(c.sm[1], cf.carrier_lock_test_smoother_alpha, -1.0F, 0.0F, cf.carrier_lock_test_smoother_samples);
    TrkHot& t = ch.h;
    t.spc = cf.early_late_space_chips;
    t.code_freq_chips = c.code_chip_rate;
    t.corr_time = c.code_period;
    sm_reset(t, 0);
    sm_reset(t, 1);
    t.state = 0;
    ch.code_filter.T = (float)c.code_period;
    ch.code_filter.bw = cf.dll_bw_hz;
    ch.code_filter.order = cf.dll_filter_order;
    lf_update(ch.code_filter);
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

// Dynamic LDS of a launch: the replica and the input window, padded up to a whole
// CU's LDS so that no workgroup of another kernel (the acquisition grid on the
// other queue) can share the CU with a tracking workgroup -- the loop is a
// latency chain and co-resident FFT waves would slow every call down.
constexpr size_t kCuLds = 160 * 1024;
constexpr size_t kStaticLdsMargin = 4 * 1024;  // the kernel's static __shared__ arrays
// Streamed calls (vector_length > kWinCore): two chunk buffers in the LDS left
// after the replicas, each (chunk + kTrkThreads + kHalo) items (a last chunk carries
// a tail of up to kTrkThreads samples) + 16 alignment bytes rounded up to whole
// glds rows; chunk a multiple of kWinCore.  chunk = 0: no room (the
// calls then read HBM directly).
int item_size(int item_type) { return item_type == GSDR_ITEM_GR_COMPLEX ? 8 : (item_type == GSDR_ITEM_CSHORT ? 4 : 2); }
int stream_buffer_bytes(int chunk, int isz) { return (((chunk + kHalo) * isz + 16) / kStreamRow + 2) * kStreamRow; }
void stream_plan(size_t lds_bytes, int code_pad, int data_pad, int isz, int& chunk, int& sbuf)
{
    const long avail = (long)lds_bytes - (long)(code_pad + data_pad) * (long)sizeof(float);
    chunk = 0;
    sbuf = 0;
    int cap = 64 * kWinCore;
    if (const char* e = std::getenv("GSDR_TRK_STREAM_CHUNK")) cap = std::max(kWinCore, std::atoi(e) / kWinCore * kWinCore);
    for (int c = kWinCore; c <= cap; c += kWinCore)
        {
            if (2L * stream_buffer_bytes(c + kTrkThreads, isz) > avail) break;
            chunk = c;
            sbuf = stream_buffer_bytes(c + kTrkThreads, isz);
        }
}

size_t lds_for(int code_pad, int data_pad)
{
    const size_t need = (size_t)(code_pad + data_pad) * sizeof(float) +
                        std::max((size_t)(kWinCore + kHalo) * sizeof(float2), (size_t)2 * stream_buffer_bytes(kWinCore + kTrkThreads, 8));
    // LDS reserved per channel workgroup: by default the whole CU, so no acquisition
    // workgroup shares its issue slots once it runs; GSDR_TRK_LDS_KB trades that for
    // an earlier start on a busy chip (a full-CU workgroup waits for an empty CU).
    size_t reserve = kCuLds - kStaticLdsMargin;
    if (const char* e = std::getenv("GSDR_TRK_LDS_KB")) reserve = std::min(reserve, (size_t)std::atoi(e) * 1024);
    return std::max(need, reserve);
}

int launch(gsdr_trk* k, const void* iq, uint64_t iq_first, uint64_t iq_items, uint32_t max_epochs, gsdr_trk_epoch* out,
    uint32_t* nout, hipStream_t s)
{
    uint64_t* timing = nullptr;
    if (k->timing_on)
        {
            const size_t need = (size_t)k->conf.max_channels * max_epochs * kTimingSlots;
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
    int chunk = 0, sbuf = 0;
    stream_plan(k->lds_bytes, k->code_pad, k->data_pad, item_size(k->conf.item_type), chunk, sbuf);
    if (k->conf.item_type == GSDR_ITEM_GR_COMPLEX)
        hipLaunchKernelGGL((trk_kernel<GSDR_ITEM_GR_COMPLEX>), grid, dim3(kTrkThreads), k->lds_bytes, s, k->d_consts, k->d_chans,
            (const float* const*)k->d_codes, (const float* const*)k->d_data_codes, iq, iq_first, iq_items, max_epochs, out,
            nout, k->code_pad, k->data_pad, timing, k->timing_wall, chunk, sbuf);
    else if (k->conf.item_type == GSDR_ITEM_CSHORT)
        hipLaunchKernelGGL((trk_kernel<GSDR_ITEM_CSHORT>), grid, dim3(kTrkThreads), k->lds_bytes, s, k->d_consts, k->d_chans,
            (const float* const*)k->d_codes, (const float* const*)k->d_data_codes, iq, iq_first, iq_items, max_epochs, out,
            nout, k->code_pad, k->data_pad, timing, k->timing_wall, chunk, sbuf);
    else
        hipLaunchKernelGGL((trk_kernel<GSDR_ITEM_IBYTE>), grid, dim3(kTrkThreads), k->lds_bytes, s, k->d_consts, k->d_chans,
            (const float* const*)k->d_codes, (const float* const*)k->d_data_codes, iq, iq_first, iq_items, max_epochs, out,
            nout, k->code_pad, k->data_pad, timing, k->timing_wall, chunk, sbuf);
    GSDR_HIP(hipGetLastError());
    GSDR_HIP(hipEventRecord(k->last_launch, s));
    if (k->profiling)
        {
            GSDR_HIP(hipEventRecord(e1, s));
            k->prof_recs.push_back({e0, e1});
        }
    if (timing)
        {
            k->timing_epochs = max_epochs;  // summarised (last launch) on destroy, no sync here
            k->timing_nout = nout;
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
    c->smoother_length = 10;
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
    GSDR_REQUIRE(conf->signal >= GSDR_SIGNAL_GPS_1C && conf->signal <= GSDR_SIGNAL_BDS_B1, GSDR_E_UNSUPPORTED,
        "gsdr_trk_create: signal %d not implemented", conf->signal);
    GSDR_REQUIRE(conf->item_type >= GSDR_ITEM_GR_COMPLEX && conf->item_type <= GSDR_ITEM_IBYTE, GSDR_E_ARG,
        "gsdr_trk_create: unknown item type %d", conf->item_type);
    GSDR_REQUIRE(conf->extend_correlation_symbols >= 1, GSDR_E_ARG,
        "gsdr_trk_create: extend_correlation_symbols must be >= 1");
    GSDR_REQUIRE(!conf->high_dyn || conf->smoother_length <= (uint32_t)kMaxSmoother, GSDR_E_UNSUPPORTED,
        "gsdr_trk_create: smoother_length %u > %d", conf->smoother_length, kMaxSmoother);
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
    // GPS L1 C/A and BeiDou B1I force track_pilot off (dll_pll_veml_tracking.cc:183, :402)
    if (k->conf.signal != GSDR_SIGNAL_GAL_1B) k->conf.track_pilot = 0;
    {
        // the adapters' vector_length = round(fs_in / (chip rate / code length))
        const SignalParams sp = signal_params(k->conf.signal);
        if (k->conf.vector_length == 0)
            k->conf.vector_length = (uint32_t)std::lround(conf->fs_in / (sp.chip_rate / (double)sp.length_chips));
    }
    const uint32_t nch = k->conf.max_channels;
    k->h_consts.resize(nch);
    k->h_chans.resize(nch);
    for (uint32_t c = 0; c < nch; ++c) init_channel(k->conf, k->h_consts[c], k->h_chans[c]);
    k->code_bufs.assign(nch, nullptr);
    k->data_code_bufs.assign(nch, nullptr);
    k->data_code_len.assign(nch, 0);
    k->code_pad = 1024 + 2 * kCodeMargin;  // grows with the longest replica started (gsdr_trk_start)
    k->data_pad = 0;
    k->lds_bytes = lds_for(k->code_pad, k->data_pad);
    if (const char* tv = std::getenv("GSDR_TRK_TIMING"))
        {
            k->timing_on = std::atoi(tv) != 0;
            k->timing_wall = std::atoi(tv) == 2;
        }
    hipError_t e = hipStreamCreateWithFlags(&k->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&k->last_launch, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc(&k->d_consts, nch * sizeof(TrkConst));
    if (e == hipSuccess) e = hipMalloc(&k->d_chans, nch * sizeof(TrkChan));
    if (e == hipSuccess) e = hipMalloc(&k->d_snap[0], nch * sizeof(TrkChan));
    if (e == hipSuccess) e = hipMalloc(&k->d_snap[1], nch * sizeof(TrkChan));
    if (e == hipSuccess) e = hipMalloc(&k->d_codes, nch * sizeof(float*));
    if (e == hipSuccess) e = hipMalloc(&k->d_nout, nch * sizeof(uint32_t));
    for (uint32_t c = 0; c < nch && e == hipSuccess; ++c) e = hipMalloc(&k->code_bufs[c], kMaxCodeFloats * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(k->d_codes, k->code_bufs.data(), nch * sizeof(float*), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMalloc(&k->d_data_codes, nch * sizeof(float*));
    if (k->conf.track_pilot)
        for (uint32_t c = 0; c < nch && e == hipSuccess; ++c)
            e = hipMalloc(&k->data_code_bufs[c], kMaxCodeFloats * sizeof(float));
    if (e == hipSuccess) e = hipMemcpy(k->d_data_codes, k->data_code_bufs.data(), nch * sizeof(float*), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(k->d_consts, k->h_consts.data(), nch * sizeof(TrkConst), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(k->d_chans, k->h_chans.data(), nch * sizeof(TrkChan), hipMemcpyHostToDevice);
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)trk_kernel<GSDR_ITEM_GR_COMPLEX>, hipFuncAttributeMaxDynamicSharedMemorySize,
            (int)(kCuLds - kStaticLdsMargin));
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)trk_kernel<GSDR_ITEM_CSHORT>, hipFuncAttributeMaxDynamicSharedMemorySize,
            (int)(kCuLds - kStaticLdsMargin));
    if (e == hipSuccess)
        e = hipFuncSetAttribute((const void*)trk_kernel<GSDR_ITEM_IBYTE>, hipFuncAttributeMaxDynamicSharedMemorySize,
            (int)(kCuLds - kStaticLdsMargin));
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
    if (k->timing_on && k->d_timing && k->timing_epochs)
        {
            const uint32_t nch = k->conf.max_channels, me = k->timing_epochs;
            std::vector<uint64_t> tm((size_t)nch * me * kTimingSlots);
            std::vector<uint32_t> cnt(nch);
            if (hipMemcpy(tm.data(), k->d_timing, tm.size() * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess &&
                hipMemcpy(cnt.data(), k->timing_nout, nch * sizeof(uint32_t), hipMemcpyDeviceToHost) == hipSuccess)
                for (uint32_t c = 0; c < nch; ++c)
                    for (uint32_t e = 0; e < cnt[c] && e < me; ++e)
                        {
                            const uint64_t* r = &tm[((size_t)c * me + e) * kTimingSlots];
                            for (int q = 0; q + 1 < kStampSlots; ++q)
                                if (r[q + 1] >= r[q]) k->tsum[q] += (double)(r[q + 1] - r[q]);
                            if (e + 1 < cnt[c] && e + 1 < me)
                                {
                                    const uint64_t next0 = tm[((size_t)c * me + e + 1) * kTimingSlots];
                                    if (next0 >= r[kStampSlots - 1]) k->tsum[kStampSlots - 1] += (double)(next0 - r[kStampSlots - 1]);
                                }
                            for (int q = kStampSlots; q < kTimingSlots; ++q) k->tsum[q] += (double)r[q];  // durations / offsets
                            k->tcount++;
                        }
        }
    if (k->timing_on && k->tcount)
        {
            static const char* names[kTimingSlots] = {"prep", "correlate", "state-load", "tap-sum", "cn0-lock", "dll-pll",
                "update-vars", "rest", "next-plan", "loop-top", "(correlate's stream-wait)", "(w2 lock-test start)",
                "(w2 lock-test end)", "(w0 at the lock join)", "(w1 EVM end)", "(w0 at the EVM join)",
                "(w0 past the EVM join)"};
            std::fprintf(stderr, "gsdr_trk timing: %llu calls, %s ticks per call:", (unsigned long long)k->tcount,
                "wall_clock64 (100 MHz)");
            for (int q = 0; q < kTimingSlots; ++q) std::fprintf(stderr, " %s %.0f", names[q], k->tsum[q] / k->tcount);
            std::fprintf(stderr, "\n");
        }
    if (k->d_timing) (void)hipFree(k->d_timing);
    for (auto& r : k->prof_recs)
        {
            (void)hipEventDestroy(r.first);
            (void)hipEventDestroy(r.second);
        }
    for (hipEvent_t e : k->prof_pool) (void)hipEventDestroy(e);
    for (auto& u : k->sub)
        {
            if (u.done)
                {
                    (void)hipEventSynchronize(u.done);
                    (void)hipEventDestroy(u.done);
                }
            if (u.h_out) (void)hipHostFree(u.h_out);
            if (u.h_nout) (void)hipHostFree(u.h_nout);
        }
    if (k->last_launch)
        {
            (void)hipEventSynchronize(k->last_launch);
            (void)hipEventDestroy(k->last_launch);
        }
    for (float* p : k->code_bufs)
        if (p) (void)hipFree(p);
    for (float* p : k->data_code_bufs)
        if (p) (void)hipFree(p);
    void* bufs[] = {k->d_consts, k->d_chans, k->d_snap[0], k->d_snap[1], k->d_codes, k->d_data_codes, k->d_nout, k->d_out,
        k->d_iq};
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
    GSDR_REQUIRE(!k->conf.track_pilot || k->data_code_len[ch] == code_samples, GSDR_E_STATE,
        "gsdr_trk_start: pilot tracking needs gsdr_trk_set_data_code with %d samples for channel %d first", code_samples,
        ch);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    // the device copy is authoritative between launches (the loop runs there)
    GSDR_HIP(hipStreamWaitEvent(k->stream, k->last_launch, 0));
    GSDR_HIP(hipMemcpyAsync(&k->h_chans[ch], k->d_chans + ch, sizeof(TrkChan), hipMemcpyDeviceToHost, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    TrkConst& c = k->h_consts[ch];
    TrkChan& tc = k->h_chans[ch];
    TrkHot& t = tc.h;
    // start_tracking (:640-882)
    c.prn = prn;
    if (k->conf.signal == GSDR_SIGNAL_BDS_B1)
        {
            uint32_t reg[5], bits[5];
            if ((prn > 0 && prn < 6) || prn > 58)
                {
                    // GEO (D2): D2 preamble search, 2 symbols per bit (:762-778)
                    c.symbols_per_bit = 2;
                    c.secondary = 0;
                    set_secondary(c, kBdsB1GeoPreamble, 22);
                    c.data_sec_len = 0;
                    c.data_sec_str = 0;
                }
            else
                {
                    // D1: NH code, wiped from the data symbols too (:779-795)
                    c.symbols_per_bit = 20;
                    c.secondary = 1;
                    set_secondary(c, kBdsB1Nh, 20);
                    code_registers(kBdsB1Nh, 20, reg, bits);
                    c.data_sec_len = 20;
                    c.data_sec_str = bits[0];
                }
        }
    c.code_samples = code_samples;
    c.acq_sample_stamp = acq_samplestamp;
    double acq_code_phase_samples = acq_delay_samples;
    t.carrier_doppler_hz = acq_doppler_hz;
    t.carrier_phase_step_rad = kTwoPi * t.carrier_doppler_hz / c.fs_in;
    t.carrier_phase_rate_step_rad = 0.0;
    t.hist_n = 0;  // d_carr_ph_history.clear(), d_code_ph_history.clear() (:651-652)
    t.hist_head = 0;
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
    set_shifts(k->conf, c);
    t.corr_time = c.code_period;  // :860
    t.narrow = 0;
    t.extend_count = 0;
    c.extend_correlation_symbols = std::max(1, k->conf.extend_correlation_symbols);  // :657
    if (k->conf.signal == GSDR_SIGNAL_BDS_B1 && ((prn > 0 && prn < 6) || prn > 58))
        c.extend_correlation_symbols = std::min(c.extend_correlation_symbols, 2);  // GEO (:775-778)
    c.corr_time_ext = (double)((float)c.extend_correlation_symbols * (float)c.code_period);  // :1949
    cf_set_params(c.cf, k->conf.fll_bw_hz, k->conf.pll_bw_hz, k->conf.pll_filter_order);
    tc.code_filter.bw = k->conf.dll_bw_hz;
    lf_update(tc.code_filter);
    tc.code_filter.T = (float)c.code_period;
    lf_update(tc.code_filter);
    // Tracking_FLL_PLL_filter::initialize (tracking_FLL_PLL_filter.cc:61-74)
    const float dop0 = (float)acq_doppler_hz;
    if (c.cf.order == 3)
        {
            t.cf_x = 2.0F * dop0;
            t.cf_w = 0;
        }
    else
        {
            t.cf_w = dop0;
            t.cf_x = 0;
        }
    lf_initialize(tc.code_filter, 0.0F);
    t.cloop = 1;
    t.pull_in_transitory = 1;
    t.circ_size = 0;
    for (int w = 0; w < 5; ++w) t.circ[w] = 0u;
    t.acc_carrier_phase_initialized = 0;
    // state 1: pull-in alignment (:1813-1844)
    const int64_t diff = (int64_t)nitems_read - (int64_t)c.acq_sample_stamp;
    const double delta = (double)diff - acq_code_phase_samples;
    t.code_freq_chips = c.code_chip_rate;
    t.code_phase_step_chips = t.code_freq_chips / c.fs_in;
    t.code_phase_rate_step_chips = 0.0;
    const double T_chip_mod = 1.0 / t.code_freq_chips;
    const double T_prn_mod = T_chip_mod * (double)c.code_length_chips;
    const double T_prn_mod_samples = T_prn_mod * c.fs_in;
    acq_code_phase_samples = T_prn_mod_samples - std::fmod(delta, T_prn_mod_samples);
    t.current_prn_length_samples = (int32_t)std::round(T_prn_mod_samples);
    const int32_t offset = (int32_t)std::round(acq_code_phase_samples);
    t.acc_carrier_phase_rad -= t.carrier_phase_step_rad * (double)offset;
    t.state = 2;
    sm_reset(t, 0);
    sm_reset(t, 1);
    t.next_sample = nitems_read + (uint64_t)(int64_t)offset;
    *first_sample = t.next_sample;
    {
        const int cp = std::max(k->code_pad, (code_samples + 2 * kCodeMargin + 1) & ~1);
        const int dp = k->conf.track_pilot ? cp : 0;
        GSDR_REQUIRE(lds_for(cp, dp) <= kCuLds - kStaticLdsMargin, GSDR_E_UNSUPPORTED,
            "gsdr_trk_start: replica of %d samples does not fit the LDS next to the input window", code_samples);
        k->code_pad = cp;
        k->data_pad = dp;
    }
    k->lds_bytes = lds_for(k->code_pad, k->data_pad);
    GSDR_HIP(hipMemcpyAsync(k->code_bufs[ch], code, (size_t)code_samples * sizeof(float), hipMemcpyHostToDevice,
        k->stream));
    GSDR_HIP(hipMemcpyAsync(k->d_consts + ch, &c, sizeof(TrkConst), hipMemcpyHostToDevice, k->stream));
    GSDR_HIP(hipMemcpyAsync(k->d_chans + ch, &tc, sizeof(TrkChan), hipMemcpyHostToDevice, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    return GSDR_OK;
}

int gsdr_trk_set_data_code(gsdr_trk* k, int ch, const float* data_code, int code_samples)
{
    GSDR_REQUIRE(k && data_code, GSDR_E_ARG, "gsdr_trk_set_data_code: null argument");
    GSDR_REQUIRE(ch >= 0 && ch < (int)k->conf.max_channels, GSDR_E_ARG, "gsdr_trk_set_data_code: channel %d", ch);
    GSDR_REQUIRE(k->conf.track_pilot, GSDR_E_STATE, "gsdr_trk_set_data_code: the handle does not track a pilot");
    GSDR_REQUIRE(code_samples >= 1 && code_samples <= kMaxCodeFloats, GSDR_E_UNSUPPORTED,
        "gsdr_trk_set_data_code: replica of %d samples outside [1,%d]", code_samples, kMaxCodeFloats);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    GSDR_HIP(hipMemcpyAsync(k->data_code_bufs[ch], data_code, (size_t)code_samples * sizeof(float),
        hipMemcpyHostToDevice, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    k->data_code_len[ch] = code_samples;
    return GSDR_OK;
}

int gsdr_trk_stop(gsdr_trk* k, int ch)
{
    GSDR_REQUIRE(k, GSDR_E_ARG, "gsdr_trk_stop: null handle");
    GSDR_REQUIRE(ch >= 0 && ch < (int)k->conf.max_channels, GSDR_E_ARG, "gsdr_trk_stop: channel %d", ch);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    const int32_t zero = 0;
    GSDR_HIP(hipStreamWaitEvent(k->stream, k->last_launch, 0));
    GSDR_HIP(hipMemcpyAsync(reinterpret_cast<char*>(k->d_chans + ch) + offsetof(TrkChan, h) + offsetof(TrkHot, state),
        &zero, sizeof(zero),
        hipMemcpyHostToDevice, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    return GSDR_OK;
}

// msg_handler_telemetry_to_trk (dll_pll_veml_tracking.cc:614-637): a telemetry fault
// sets d_carrier_lock_fail_counter = 200000, so the next lock check that evaluates the
// counters (states 2 / 4 with a full CN0 buffer, :986-1024) reports the loss of lock.
// Written into the channel's device state between launches, like gsdr_trk_stop.
int gsdr_trk_force_loss_of_lock(gsdr_trk* k, int ch)
{
    GSDR_REQUIRE(k, GSDR_E_ARG, "gsdr_trk_force_loss_of_lock: null handle");
    GSDR_REQUIRE(ch >= 0 && ch < (int)k->conf.max_channels, GSDR_E_ARG, "gsdr_trk_force_loss_of_lock: channel %d", ch);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    const int32_t forced = 200000;
    GSDR_HIP(hipStreamWaitEvent(k->stream, k->last_launch, 0));
    GSDR_HIP(hipMemcpyAsync(reinterpret_cast<char*>(k->d_chans + ch) + offsetof(TrkChan, h) +
                                offsetof(TrkHot, carrier_lock_fail_counter),
        &forced, sizeof(forced), hipMemcpyHostToDevice, k->stream));
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

int gsdr_trk_run_stream(gsdr_trk* k, gsdr_stream* ring, uint32_t max_epochs, gsdr_trk_epoch* out_dev,
    uint32_t* n_out_dev, void* stream)
{
    GSDR_REQUIRE(k && ring && out_dev && n_out_dev, GSDR_E_ARG, "gsdr_trk_run_stream: null argument");
    GSDR_REQUIRE(gsdr::stream_item_type(ring) == k->conf.item_type, GSDR_E_ARG,
        "gsdr_trk_run_stream: ring item type %d != tracking item type %d", gsdr::stream_item_type(ring),
        k->conf.item_type);
    GSDR_REQUIRE(gsdr::stream_device(ring) == k->device, GSDR_E_ARG,
        "gsdr_trk_run_stream: ring on device %d, tracking handle on device %d", gsdr::stream_device(ring), k->device);
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    hipStream_t s = stream ? (hipStream_t)stream : k->stream;
    gsdr::StreamReader rd(ring);  // ring lock from window choice to reader-event record
    uint64_t first = 0, n = 0;
    int rc = rd.span(&first, &n);
    if (rc != GSDR_OK) return rc;
    const void* iq = nullptr;
    rc = rd.view(first, n, &iq);
    if (rc != GSDR_OK) return rc;
    rc = rd.acquire(s);
    if (rc != GSDR_OK) return rc;
    rc = launch(k, iq, first, n, max_epochs, out_dev, n_out_dev, s);
    if (rc != GSDR_OK) return rc;
    return rd.release(s);
}

int gsdr_trk_run_stream_host(gsdr_trk* k, gsdr_stream* ring, uint32_t max_epochs, gsdr_trk_epoch* out_host,
    uint32_t* n_out_host)
{
    GSDR_REQUIRE(k && ring && out_host && n_out_host, GSDR_E_ARG, "gsdr_trk_run_stream_host: null argument");
    {
        std::lock_guard<std::mutex> lk(k->mu);
        gsdr::DeviceGuard g(k->device);
        int rc = ensure_out(k, max_epochs);
        if (rc != GSDR_OK) return rc;
    }
    int rc = gsdr_trk_run_stream(k, ring, max_epochs, k->d_out, k->d_nout, nullptr);
    if (rc != GSDR_OK) return rc;
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    GSDR_HIP(hipMemcpyAsync(n_out_host, k->d_nout, k->conf.max_channels * sizeof(uint32_t), hipMemcpyDeviceToHost,
        k->stream));
    GSDR_HIP(hipMemcpyAsync(out_host, k->d_out, (size_t)k->conf.max_channels * max_epochs * sizeof(gsdr_trk_epoch),
        hipMemcpyDeviceToHost, k->stream));
    GSDR_HIP(hipStreamSynchronize(k->stream));
    return GSDR_OK;
}

int gsdr_trk_submit_stream(gsdr_trk* k, gsdr_stream* ring, uint32_t max_epochs)
{
    GSDR_REQUIRE(k && ring, GSDR_E_ARG, "gsdr_trk_submit_stream: null argument");
    GSDR_REQUIRE(max_epochs >= 1, GSDR_E_ARG, "gsdr_trk_submit_stream: max_epochs must be >= 1");
    std::lock_guard<std::mutex> submit_lk(k->submit_mu);
    gsdr_trk::Submission* u = nullptr;
    {
        std::lock_guard<std::mutex> lk(k->mu);
        GSDR_REQUIRE(k->sub_count < gsdr_trk::kSubmissions, GSDR_E_STATE,
            "gsdr_trk_submit_stream: %d submissions in flight, collect the oldest first", gsdr_trk::kSubmissions);
        gsdr::DeviceGuard g(k->device);
        const uint32_t nch = k->conf.max_channels;
        u = &k->sub[(k->sub_head + k->sub_count) % gsdr_trk::kSubmissions];
        if (max_epochs > u->cap)
            {
                // not pending: nothing in flight writes this slot's buffer
                if (u->h_out) GSDR_HIP(hipHostFree(u->h_out));
                u->h_out = nullptr;
                u->cap = 0;
                GSDR_HIP(hipHostMalloc(reinterpret_cast<void**>(&u->h_out), (size_t)nch * max_epochs * sizeof(gsdr_trk_epoch),
                    hipHostMallocMapped));
                u->cap = max_epochs;
            }
        if (!u->h_nout)
            {
                GSDR_HIP(hipHostMalloc(reinterpret_cast<void**>(&u->h_nout), nch * sizeof(uint32_t), hipHostMallocMapped));
                GSDR_HIP(hipEventCreateWithFlags(&u->done, hipEventDisableTiming));
            }
    }
    // on the handle's stream: ordered after the submissions still in flight; the
    // kernel's records land in the pinned host buffers themselves
    int rc = gsdr_trk_run_stream(k, ring, max_epochs, u->h_out, u->h_nout, nullptr);
    if (rc != GSDR_OK) return rc;
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    GSDR_HIP(hipEventRecord(u->done, k->stream));
    u->epochs = max_epochs;
    k->sub_count++;
    return GSDR_OK;
}

int gsdr_trk_collect(gsdr_trk* k, int wait, gsdr_trk_epoch* out_host, uint32_t* n_out_host, uint32_t* max_epochs)
{
    GSDR_REQUIRE(k && out_host && n_out_host, GSDR_E_ARG, "gsdr_trk_collect: null argument");
    std::lock_guard<std::mutex> lk(k->mu);
    GSDR_REQUIRE(k->sub_count > 0, GSDR_E_STATE, "gsdr_trk_collect: nothing submitted");
    gsdr::DeviceGuard g(k->device);
    gsdr_trk::Submission& u = k->sub[k->sub_head];
    if (!wait)
        {
            const hipError_t q = hipEventQuery(u.done);
            if (q == hipErrorNotReady) return 1;
            GSDR_HIP(q);
        }
    else
        GSDR_HIP(hipEventSynchronize(u.done));
    k->sub_head = (k->sub_head + 1) % gsdr_trk::kSubmissions;
    k->sub_count--;
    const uint32_t nch = k->conf.max_channels, me = u.epochs;
    std::memcpy(n_out_host, u.h_nout, nch * sizeof(uint32_t));
    // each channel's records only (a few of max_epochs per advance)
    for (uint32_t c = 0; c < nch; ++c)
        std::memcpy(out_host + (size_t)c * me, u.h_out + (size_t)c * me, std::min(u.h_nout[c], me) * sizeof(gsdr_trk_epoch));
    if (max_epochs) *max_epochs = me;
    return GSDR_OK;
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
    GSDR_HIP(hipStreamWaitEvent(k->stream, k->last_launch, 0));
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

int gsdr_trk_set_cu_mask(gsdr_trk* k, const uint32_t* mask, int n_words)
{
    GSDR_REQUIRE(k, GSDR_E_ARG, "gsdr_trk_set_cu_mask: null handle");
    std::lock_guard<std::mutex> lk(k->mu);
    gsdr::DeviceGuard g(k->device);
    return gsdr::replace_stream(&k->stream, mask, n_words);
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
