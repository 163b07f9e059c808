/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of GNSS-SDR's DLL/PLL tracking channel, dll_pll_veml_tracking
 * (src/algorithms/tracking/gnuradio_blocks/dll_pll_veml_tracking.cc), for GPS
 * L1 C/A, Galileo E1 (VEML, pilot or data tracking) and BeiDou B1I (D1 NH code,
 * D2 GEO preamble), together with the library pieces it calls:
 *   Tracking_loop_filter        src/algorithms/tracking/libs/tracking_loop_filter.cc:20-267
 *   Tracking_FLL_PLL_filter     src/algorithms/tracking/libs/tracking_FLL_PLL_filter.cc:23-101
 *   discriminators              src/algorithms/tracking/libs/tracking_discriminators.cc:25-149
 *   cn0_m2m4_estimator,
 *   carrier_lock_detector       src/algorithms/tracking/libs/lock_detectors.cc:90-148
 *   Exponential_Smoother        src/algorithms/tracking/libs/exponential_smoother.cc:23-110
 * and, for the correlation step, this directory's restatement of the VOLK-GNSSSDR
 * generic resampler + rotator (volk_oracle.c, orc_multicorrelator_real_codes).
 *
 * Only tests/ (and bench.py's cpu_baseline leg) load it, as the checker.  The
 * float/double types of every expression follow the reference member and local
 * types (dll_pll_veml_tracking.h:117-209, the loop-filter headers), built with
 * -ffp-contract=off like the reference's x86-64 build (no FMA contraction).
 *
 * gr::fast_atan2f (GNU Radio, behind pll_four_quadrant_atan, tracking_discriminators.cc:86-89;
 * GNU Radio's version is not pinned by the reference and its source is not in the
 * tree) is restated as atan2f -- its table/polynomial approximations stay within
 * ~1e-6 rad of it.
 *
 * Pinning: the loop filters and the E-L discriminator are checked against the
 * reference's own unit-test expectations (tracking_loop_filter_test.cc,
 * discriminator_test.cc) in tests/test_oracle_tracking.py; the channel state
 * machine itself has no numeric golden vector in the reference (its tracking
 * tests need GNU Radio and recorded captures) — "parity unpinned" beyond this
 * line-by-line restatement.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gsdr.h"

typedef struct
{
    float re, im;
} tcf;

/* MATH_CONSTANTS.h:47-50 (GNSS_PI as defined for GNSS, not M_PI) */
#define GNSS_PI_REF 3.1415926535898
#define TWO_PI_REF (2.0 * GNSS_PI_REF)
#define HALF_PI_REF (GNSS_PI_REF / 2.0)

/* GPS_L1_CA.h:34-73 */
#define GPS_L1_FREQ_HZ_REF 1.57542e9
#define GPS_L1_CA_CODE_RATE_CPS_REF 1.023e6
#define GPS_L1_CA_CODE_PERIOD_S_REF 0.001
#define GPS_L1_CA_CODE_LENGTH_CHIPS_REF 1023
#define GPS_CA_PREAMBLE_LENGTH_SYMBOLS_REF 160
#define GPS_CA_TELEMETRY_SYMBOLS_PER_BIT_REF 20
static const char GPS_CA_PREAMBLE_SYMBOLS_STR_REF[161] =
    "1111111111111111111100000000000000000000000000000000000000000000000000000000000011111111111111111111000000000000"
    "000000001111111111111111111111111111111111111111";

/* Galileo_E1.h:32-52 */
#define GALILEO_E1_FREQ_HZ_REF 1.57542e9
#define GALILEO_E1_CODE_CHIP_RATE_CPS_REF 1.023e6
#define GALILEO_E1_CODE_PERIOD_S_REF 0.004
#define GALILEO_E1_B_CODE_LENGTH_CHIPS_REF 4092
#define GALILEO_E1_C_SECONDARY_CODE_LENGTH_REF 25
static const char GALILEO_E1_C_SECONDARY_CODE_REF[26] = "0011100000001010110110010";

/* Beidou_B1I.h:30-48 */
#define BEIDOU_B1I_FREQ_HZ_REF 1.561098e9
#define BEIDOU_B1I_CODE_RATE_CPS_REF 2.046e6
#define BEIDOU_B1I_CODE_PERIOD_S_REF 0.001
#define BEIDOU_B1I_CODE_LENGTH_CHIPS_REF 2046
#define BEIDOU_B1I_SECONDARY_CODE_LENGTH_REF 20
#define BEIDOU_B1I_TELEMETRY_SYMBOLS_PER_BIT_REF 20
#define BEIDOU_B1I_GEO_TELEMETRY_SYMBOLS_PER_BIT_REF 2
#define BEIDOU_B1I_GEO_PREAMBLE_LENGTH_SYMBOLS_REF 22
static const char BEIDOU_B1I_SECONDARY_CODE_STR_REF[21] = "00000100110101001110";
static const char BEIDOU_B1I_GEO_PREAMBLE_SYMBOLS_STR_REF[23] = "1111110000001100001100";

void orc_multicorrelator_real_codes(float* out, const float* sig, const float* code, unsigned int L,
    const float* shifts, int K, float rem_carr, float carr_step, float carr_rate, float rem_code, float code_step,
    float code_rate, unsigned int N, int high_dyn, int assoc);

/* ------------------------------------------------------------------------ */
/* Tracking_loop_filter                                                      */
/* ------------------------------------------------------------------------ */
#define LF_HIST 4 /* MAX_LOOP_HISTORY_LENGTH */
typedef struct
{
    float inputs[LF_HIST], outputs[LF_HIST];
    float icoef[4], ocoef[3];
    int nin, nout;
    float bw, T;
    int order, idx, last_int;
} lf_t;

/* tracking_loop_filter.cc:98-197 (float members, double literals as written) */
static void lf_update(lf_t* f)
{
    float g1, g2, g3, wn;
    const float T = f->T;
    const float zeta = 1.0F / sqrtf(2.0F);
    switch (f->order)
        {
        case 1:
            wn = f->bw * 4.0F;
            g1 = wn;
            if (f->last_int)
                {
                    f->nin = 2;
                    f->icoef[0] = (float)(g1 * T / 2.0);
                    f->icoef[1] = (float)(g1 * T / 2.0);
                    f->nout = 1;
                    f->ocoef[0] = 1.0F;
                }
            else
                {
                    f->nin = 1;
                    f->icoef[0] = g1;
                    f->nout = 0;
                }
            break;
        case 2:
            wn = f->bw * (8.0F * zeta) / (4.0F * zeta * zeta + 1.0F);
            g1 = wn * wn;
            g2 = wn * 2.0F * zeta;
            if (f->last_int)
                {
                    f->nin = 3;
                    f->icoef[0] = (float)(T / 2.0 * (g1 * T / 2.0 + g2));
                    f->icoef[1] = (float)(T * T / 2.0 * g1);
                    f->icoef[2] = (float)(T / 2.0 * (g1 * T / 2.0 - g2));
                    f->nout = 2;
                    f->ocoef[0] = 2.0F;
                    f->ocoef[1] = -1.0F;
                }
            else
                {
                    f->nin = 2;
                    f->icoef[0] = (float)(g1 * T / 2.0 + g2);
                    f->icoef[1] = (float)(g1 * T / 2.0 - g2);
                    f->nout = 1;
                    f->ocoef[0] = 1.0F;
                }
            break;
        default:
            {
                wn = f->bw / 0.7845F;
                const float a3 = 1.1F;
                const float b3 = 2.4F;
                g1 = wn * wn * wn;
                g2 = a3 * wn * wn;
                g3 = b3 * wn;
                if (f->last_int)
                    {
                        f->nin = 4;
                        f->icoef[0] = (float)(T / 2.0 * (g3 + T / 2.0 * (g2 + T / 2.0 * g1)));
                        f->icoef[1] = (float)(T / 2.0 * (-g3 + T / 2.0 * (g2 + 3.0 * T / 2.0 * g1)));
                        f->icoef[2] = (float)(T / 2.0 * (-g3 - T / 2.0 * (g2 - 3.0 * T / 2.0 * g1)));
                        f->icoef[3] = (float)(T / 2.0 * (g3 - T / 2.0 * (g2 - T / 2.0 * g1)));
                        f->nout = 3;
                        f->ocoef[0] = 3.0F;
                        f->ocoef[1] = -3.0F;
                        f->ocoef[2] = 1.0F;
                    }
                else
                    {
                        f->nin = 3;
                        f->icoef[0] = (float)(g3 + T / 2.0 * (g2 + T / 2.0 * g1));
                        f->icoef[1] = (float)(g1 * T * T / 2.0 - 2.0 * g3);
                        f->icoef[2] = (float)(g3 + T / 2.0 * (-g2 + T / 2.0 * g1));
                        f->nout = 2;
                        f->ocoef[0] = 2.0F;
                        f->ocoef[1] = -1.0F;
                    }
            }
            break;
        }
}

/* constructor (tracking_loop_filter.cc:26-40) */
static void lf_init(lf_t* f, float T, float bw, int order, int last_int)
{
    memset(f, 0, sizeof(*f));
    f->T = T;
    f->bw = bw;
    f->order = order;
    f->last_int = last_int;
    f->idx = 0;
    lf_update(f);
}

/* initialize (:258-263) */
static void lf_initialize(lf_t* f, float initial_output)
{
    for (int i = 0; i < LF_HIST; ++i)
        {
            f->inputs[i] = 0.0F;
            f->outputs[i] = initial_output;
        }
    f->idx = LF_HIST - 1;
}

/* apply (:58-93) */
static float lf_apply(lf_t* f, float in)
{
    float result = 0.0F;
    for (int ii = 0; ii < f->nout; ++ii) result += f->ocoef[ii] * f->outputs[(f->idx + ii) % LF_HIST];
    f->idx--;
    if (f->idx < 0) f->idx += LF_HIST;
    f->inputs[f->idx] = in;
    for (int ii = 0; ii < f->nin; ++ii) result += f->icoef[ii] * f->inputs[(f->idx + ii) % LF_HIST];
    f->outputs[f->idx] = result;
    return result;
}

/* ------------------------------------------------------------------------ */
/* Tracking_FLL_PLL_filter (tracking_FLL_PLL_filter.cc:23-101)               */
/* ------------------------------------------------------------------------ */
typedef struct
{
    float w, w0p3, w0f2, x, a2, w0f, a3, w0p2, b3, w0p;
    int order;
} pll_t;

static void pll_set_params(pll_t* p, float fll_bw_hz, float pll_bw_hz, int order)
{
    p->order = order;
    if (order == 3)
        {
            p->b3 = 2.400F;
            p->a3 = 1.100F;
            p->a2 = 1.414F;
            p->w0p = pll_bw_hz / 0.7845F;
            p->w0p2 = p->w0p * p->w0p;
            p->w0p3 = p->w0p2 * p->w0p;
            p->w0f = fll_bw_hz / 0.53F;
            p->w0f2 = p->w0f * p->w0f;
        }
    else
        {
            p->a2 = 1.414F;
            p->w0p = pll_bw_hz / 0.53F;
            p->w0p2 = p->w0p * p->w0p;
            p->w0f = fll_bw_hz / 0.25F;
        }
}

static void pll_initialize(pll_t* p, float acq_doppler_hz)
{
    if (p->order == 3)
        {
            p->x = 2.0F * acq_doppler_hz;
            p->w = 0;
        }
    else
        {
            p->w = acq_doppler_hz;
            p->x = 0;
        }
}

static float pll_get_carrier_error(pll_t* p, float fll, float pll, float t)
{
    float e;
    if (p->order == 3)
        {
            p->w = p->w + t * (p->w0p3 * pll + p->w0f2 * fll);
            p->x = p->x + t * (0.5F * p->w + p->a2 * p->w0f * fll + p->a3 * p->w0p2 * pll);
            e = 0.5F * p->x + p->b3 * p->w0p * pll;
        }
    else
        {
            const float w_new = p->w + pll * p->w0p2 * t + fll * p->w0f * t;
            e = 0.5F * (w_new + p->w) + p->a2 * p->w0p * pll;
            p->w = w_new;
        }
    return e;
}

/* ------------------------------------------------------------------------ */
/* Exponential_Smoother (exponential_smoother.cc:23-110)                     */
/* ------------------------------------------------------------------------ */
#define SM_MAX_INIT 4096
typedef struct
{
    float alpha, one_minus_alpha, old, min_value, offset;
    int samples_init, counter, initializing, nbuf;
    float buf[SM_MAX_INIT];
} sm_t;

static void sm_init(sm_t* s)
{
    s->alpha = 0.001F;
    s->one_minus_alpha = 0.999F;
    s->old = 0.0F;
    s->min_value = 25.0F;
    s->offset = 12.0F;
    s->samples_init = 200;
    s->counter = 0;
    s->initializing = 1;
    s->nbuf = 0;
}

static void sm_set_alpha(sm_t* s, float a)
{
    s->alpha = a;
    if (s->alpha < 0) s->alpha = 0;
    if (s->alpha > 1) s->alpha = 1;
    s->one_minus_alpha = 1.0F - s->alpha;
}

static void sm_set_samples(sm_t* s, int n)
{
    if (n <= 0) n = 1;
    if (n > SM_MAX_INIT) n = SM_MAX_INIT;
    s->samples_init = n;
}

static void sm_reset(sm_t* s)
{
    s->initializing = 1;
    s->counter = 0;
    s->nbuf = 0;
}

static float sm_smooth(sm_t* s, float raw)
{
    float v;
    if (s->initializing)
        {
            s->counter++;
            v = raw;
            s->buf[s->nbuf++] = v;
            if (s->counter == s->samples_init)
                {
                    float acc = 0.0F;
                    for (int i = 0; i < s->nbuf; ++i) acc = acc + s->buf[i];
                    s->old = acc / (float)s->nbuf;
                    if (s->old < (s->min_value + s->offset))
                        {
                            s->counter = 0;
                            s->nbuf = 0;
                        }
                    else
                        {
                            s->initializing = 0;
                        }
                }
        }
    else
        {
            v = s->alpha * raw + s->one_minus_alpha * s->old;
            s->old = v;
        }
    return v;
}

/* ------------------------------------------------------------------------ */
/* discriminators and lock detectors                                         */
/* ------------------------------------------------------------------------ */
static double phase_unwrap(double p)
{
    if (p >= HALF_PI_REF) return p - GNSS_PI_REF;
    if (p <= -HALF_PI_REF) return p + GNSS_PI_REF;
    return p;
}

/* fll_diff_atan (tracking_discriminators.cc:62-70): std::atan on float operands */
static double fll_diff_atan(tcf s1, tcf s2, double t1, double t2)
{
    double d = (double)(atanf(s2.im / s2.re) - atanf(s1.im / s1.re));
    if (isnan(d)) d = 0;
    return phase_unwrap(d) / (t2 - t1);
}

/* pll_cloop_two_quadrant_atan (:92-99) */
static double pll_cloop_two_quadrant_atan(tcf p)
{
    if (p.re != 0.0F) return (double)atanf(p.im / p.re);
    return 0.0;
}

/* dll_nc_e_minus_l_normalized (:110-120); std::abs(complex<float>) = hypotf */
/* pll_four_quadrant_atan (tracking_discriminators.cc:86-89), fast_atan2f -> atan2f */
static double pll_four_quadrant_atan(tcf p) { return (double)atan2f(p.im, p.re); }

/* dll_nc_vemlp_normalized (tracking_discriminators.cc:139-149) */
double orc_dll_nc_vemlp_normalized(tcf ve, tcf e, tcf l, tcf vl)
{
    const double Early = sqrt(ve.re * ve.re + ve.im * ve.im + e.re * e.re + e.im * e.im);
    const double Late = sqrt(l.re * l.re + l.im * l.im + vl.re * vl.re + vl.im * vl.im);
    const double E_plus_L = Early + Late;
    if (E_plus_L == 0.0) return 0.0;
    return (Early - Late) / E_plus_L;
}

double orc_dll_nc_e_minus_l_normalized(float ere, float eim, float lre, float lim, float spc, float slope,
    float y_intercept)
{
    const double pe = (double)hypotf(ere, eim);
    const double pl = (double)hypotf(lre, lim);
    const double epl = pe + pl;
    if (epl == 0.0) return 0.0;
    return (double)((y_intercept - slope * spc) / slope) * (pe - pl) / epl;
}

/* cn0_m2m4_estimator (lock_detectors.cc:90-120) */
static float cn0_m2m4(const tcf* b, int length, float coh)
{
    float snr, psig = 0.0F, m2 = 0.0F, m4 = 0.0F, aux;
    const float n = (float)length;
    for (int i = 0; i < length; i++)
        {
            psig += fabsf(b[i].re);
            aux = b[i].im * b[i].im + b[i].re * b[i].re;
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

/* carrier_lock_detector (:133-148) */
static float carrier_lock_detector(const tcf* b, int length)
{
    float si = 0.0F, sq = 0.0F;
    for (int i = 0; i < length; i++)
        {
            si += b[i].re;
            sq += b[i].im;
        }
    const float nbp = si * si + sq * sq;
    const float nbd = si * si - sq * sq;
    return nbd / nbp;
}

/* ------------------------------------------------------------------------ */
/* the channel                                                               */
/* ------------------------------------------------------------------------ */
#define MAX_CN0_SAMPLES 1024
#define MAX_CODE 16384

typedef struct orc_trk
{
    gsdr_trk_conf p;
    /* signal (dll_pll_veml_tracking.cc:170-191) */
    double signal_carrier_freq, code_period, code_chip_rate;
    int32_t code_length_chips, code_samples_per_chip, symbols_per_bit;
    uint32_t secondary_code_length, data_secondary_code_length;
    const char* secondary_code_string;
    const char* data_secondary_code_string;
    int secondary, veml, track_pilot;
    int extend, extend_count, enable_ext; /* d_extend_correlation_symbols(_count), d_enable_extended_integration */
    int iE, iP, iL; /* tap slots of Early / Prompt / Late (VEML: VE 0, VL 4) */
    int n_taps;
    float shifts[5];
    float code[MAX_CODE];
    int code_samples;
    float data_code[MAX_CODE];
    int data_code_samples;
    tcf prompt_data;
    /* loop objects */
    sm_t cn0_smoother, lock_smoother;
    lf_t code_filter;
    pll_t carrier_filter;
    /* state (dll_pll_veml_tracking.h:117-209) */
    double acq_code_phase_samples, acq_carrier_doppler_hz, current_correlation_time_s;
    double carr_phase_error_hz, carr_freq_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips;
    double code_freq_chips, carrier_doppler_hz, acc_carrier_phase_rad, rem_code_phase_chips;
    double T_chip_seconds, T_prn_seconds, T_prn_samples, K_blk_samples;
    double carrier_lock_test, CN0_SNV_dB_Hz, carrier_lock_threshold;
    double carrier_phase_step_rad, carrier_phase_rate_step_rad, code_phase_step_chips, code_phase_rate_step_chips;
    double rem_code_phase_samples, EVM;
    tcf taps[5];
    tcf VE_accu, E_accu, P_accu, P_accu_old, L_accu, VL_accu, P_data_accu;
    tcf prompt_buffer[MAX_CN0_SAMPLES];
    tcf circ[GPS_CA_PREAMBLE_LENGTH_SYMBOLS_REF]; /* capacity secondary_code_length <= 160 */
    int circ_size, circ_head;
    uint64_t acq_sample_stamp;
    float rem_carr_phase_rad;
    float spc;
    int32_t state, current_prn_length_samples, current_symbol, current_data_symbol, cn0_estimation_counter;
    int32_t carrier_lock_fail_counter, code_lock_fail_counter;
    int pull_in_transitory, cloop, acc_carrier_phase_initialized, flag_pll_180;
    int assoc;
    /* high_dyn: d_carr_ph_history / d_code_ph_history, boost::circular_buffer of
       capacity 2*smoother_length (:554-563), element [k] counted from the oldest */
    double hc_step[64], hc_samples[64], hk_step[64], hk_samples[64];
    int hc_n, hc_head, hk_n, hk_head;
} orc_trk;

/* Dll_Pll_Conf defaults (dll_pll_conf.h:38-84, dll_pll_conf.cc:25-35 with the
 * gflags defaults of gnss_sdr_flags.cc:45-54). */
void orc_trk_conf_default(gsdr_trk_conf* c)
{
    memset(c, 0, sizeof(*c));
    c->fs_in = 2000000.0;
    c->carrier_lock_th = 0.7;
    c->vector_length = 0;
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
    c->enable_fll_pull_in = 0;
    c->enable_fll_steady_state = 0;
    c->carrier_aiding = 1;
    c->high_dyn = 0;
    c->track_pilot = 1;
    c->smoother_length = 10;
}

/* constructor (dll_pll_veml_tracking.cc:85-560) and the signal table (:170-430) */
orc_trk* orc_trk_create(const gsdr_trk_conf* conf)
{
    if (conf->signal < GSDR_SIGNAL_GPS_1C || conf->signal > GSDR_SIGNAL_BDS_B1 || conf->extend_correlation_symbols < 1 ||
        (conf->high_dyn && conf->smoother_length > 32) || conf->cn0_samples > MAX_CN0_SAMPLES || conf->cn0_samples < 1)
        return NULL;
    orc_trk* t = (orc_trk*)calloc(1, sizeof(orc_trk));
    if (!t) return NULL;
    t->p = *conf;
    t->data_secondary_code_length = 0;
    t->data_secondary_code_string = "";
    if (conf->signal == GSDR_SIGNAL_GPS_1C)
        {
            t->signal_carrier_freq = GPS_L1_FREQ_HZ_REF;
            t->code_period = GPS_L1_CA_CODE_PERIOD_S_REF;
            t->code_chip_rate = GPS_L1_CA_CODE_RATE_CPS_REF;
            t->code_samples_per_chip = 1;
            t->code_length_chips = GPS_L1_CA_CODE_LENGTH_CHIPS_REF;
            t->secondary = 0;
            t->p.track_pilot = 0;
            t->secondary_code_length = GPS_CA_PREAMBLE_LENGTH_SYMBOLS_REF;
            t->secondary_code_string = GPS_CA_PREAMBLE_SYMBOLS_STR_REF;
            t->symbols_per_bit = GPS_CA_TELEMETRY_SYMBOLS_PER_BIT_REF;
        }
    else if (conf->signal == GSDR_SIGNAL_GAL_1B)
        {
            t->signal_carrier_freq = GALILEO_E1_FREQ_HZ_REF;
            t->code_period = GALILEO_E1_CODE_PERIOD_S_REF;
            t->code_chip_rate = GALILEO_E1_CODE_CHIP_RATE_CPS_REF;
            t->code_length_chips = GALILEO_E1_B_CODE_LENGTH_CHIPS_REF;
            t->symbols_per_bit = 1;
            t->code_samples_per_chip = 2;
            t->veml = 1;
            t->secondary = t->p.track_pilot ? 1 : 0;
            t->secondary_code_length = t->secondary ? GALILEO_E1_C_SECONDARY_CODE_LENGTH_REF : 0;
            t->secondary_code_string = t->secondary ? GALILEO_E1_C_SECONDARY_CODE_REF : "";
        }
    else
        {
            t->signal_carrier_freq = BEIDOU_B1I_FREQ_HZ_REF;
            t->code_period = BEIDOU_B1I_CODE_PERIOD_S_REF;
            t->code_chip_rate = BEIDOU_B1I_CODE_RATE_CPS_REF;
            t->code_length_chips = BEIDOU_B1I_CODE_LENGTH_CHIPS_REF;
            t->symbols_per_bit = BEIDOU_B1I_TELEMETRY_SYMBOLS_PER_BIT_REF;
            t->code_samples_per_chip = 1;
            t->secondary = 1;
            t->p.track_pilot = 0;
            t->secondary_code_length = BEIDOU_B1I_SECONDARY_CODE_LENGTH_REF;
            t->secondary_code_string = BEIDOU_B1I_SECONDARY_CODE_STR_REF;
            t->data_secondary_code_length = BEIDOU_B1I_SECONDARY_CODE_LENGTH_REF;
            t->data_secondary_code_string = BEIDOU_B1I_SECONDARY_CODE_STR_REF;
        }
    t->track_pilot = t->p.track_pilot;
    /* :511-520 */
    t->enable_ext = t->p.extend_correlation_symbols > 1;
    if (!t->enable_ext) t->p.extend_correlation_symbols = 1;
    t->extend = t->p.extend_correlation_symbols;
    /* adapters: vector_length = round(fs_in / (chip rate / code length)) */
    if (t->p.vector_length == 0)
        t->p.vector_length = (uint32_t)lround(t->p.fs_in / (t->code_chip_rate / (double)t->code_length_chips));
    t->spc = t->p.early_late_space_chips; /* d_trk_parameters.spc */
    t->carrier_lock_threshold = t->p.carrier_lock_th;
    t->code_freq_chips = t->code_chip_rate;
    lf_init(&t->code_filter, (float)t->code_period, t->p.dll_bw_hz, t->p.dll_filter_order, 0);
    pll_set_params(&t->carrier_filter, t->p.fll_bw_hz, t->p.pll_bw_hz, t->p.pll_filter_order);
    if (t->veml)
        {
            t->n_taps = 5;
            t->iE = 1, t->iP = 2, t->iL = 3;
        }
    else
        {
            t->n_taps = 3;
            t->iE = 0, t->iP = 1, t->iL = 2;
        }
    sm_init(&t->cn0_smoother);
    sm_set_alpha(&t->cn0_smoother, t->p.cn0_smoother_alpha);
    sm_set_samples(&t->cn0_smoother, t->p.cn0_smoother_samples / (int)(t->code_period * 1000.0));
    sm_init(&t->lock_smoother);
    sm_set_alpha(&t->lock_smoother, t->p.carrier_lock_test_smoother_alpha);
    t->lock_smoother.min_value = -1.0F;
    t->lock_smoother.offset = 0.0F;
    sm_set_samples(&t->lock_smoother, t->p.carrier_lock_test_smoother_samples);
    t->state = 0;
    t->assoc = GSDR_ASSOC_AVX;
    return t;
}

/* the data component's replica (pilot tracking) */
int orc_trk_set_data_code(orc_trk* t, const float* code, int code_samples)
{
    if (code_samples < 1 || code_samples > MAX_CODE) return -1;
    memcpy(t->data_code, code, sizeof(float) * (size_t)code_samples);
    t->data_code_samples = code_samples;
    return 0;
}

void orc_trk_destroy(orc_trk* t) { free(t); }

void orc_trk_set_assoc(orc_trk* t, int assoc) { t->assoc = assoc; }

/* clear_tracking_vars (:1192-1213) */
static void clear_tracking_vars(orc_trk* t)
{
    for (int k = 0; k < t->n_taps; ++k) t->taps[k] = (tcf){0.0F, 0.0F};
    if (t->track_pilot)
        {
            t->prompt_data = (tcf){0.0F, 0.0F};
            t->P_data_accu = (tcf){0.0F, 0.0F};
        }
    t->P_accu_old = (tcf){0.0F, 0.0F};
    t->carr_phase_error_hz = 0.0;
    t->carr_freq_error_hz = 0.0;
    t->carr_error_filt_hz = 0.0;
    t->code_error_chips = 0.0;
    t->code_error_filt_chips = 0.0;
    t->current_symbol = 0;
    t->current_data_symbol = 0;
    t->circ_size = 0;
    t->circ_head = 0;
    t->carrier_phase_rate_step_rad = 0.0;
    t->code_phase_rate_step_chips = 0.0;
    t->hc_n = t->hc_head = t->hk_n = t->hk_head = 0;
}

/* start_tracking (:640-882) + the state-1 pull-in call (:1813-1844) at nitems_read */
int orc_trk_start(orc_trk* t, uint32_t prn, const float* code, int code_samples, double acq_delay_samples,
    double acq_doppler_hz, uint64_t acq_samplestamp, uint64_t nitems_read, uint64_t* first_sample)
{
    if (code_samples < 1 || code_samples > MAX_CODE) return -1;
    if (t->track_pilot && t->data_code_samples < 1) return -1;
    t->extend = t->p.extend_correlation_symbols; /* :657 */
    t->extend_count = 0;
    if (t->p.signal == GSDR_SIGNAL_BDS_B1)
        {
            if ((prn > 0 && prn < 6) || prn > 58)
                {
                    if (t->extend > BEIDOU_B1I_GEO_TELEMETRY_SYMBOLS_PER_BIT_REF)
                        t->extend = BEIDOU_B1I_GEO_TELEMETRY_SYMBOLS_PER_BIT_REF; /* :775-778 */
                    /* GEO (D2): preamble search, 2 symbols per bit (:762-778) */
                    t->symbols_per_bit = BEIDOU_B1I_GEO_TELEMETRY_SYMBOLS_PER_BIT_REF;
                    t->secondary = 0;
                    t->secondary_code_length = BEIDOU_B1I_GEO_PREAMBLE_LENGTH_SYMBOLS_REF;
                    t->secondary_code_string = BEIDOU_B1I_GEO_PREAMBLE_SYMBOLS_STR_REF;
                    t->data_secondary_code_length = 0;
                }
            else
                {
                    /* D1: NH code on the data (:779-795) */
                    t->symbols_per_bit = BEIDOU_B1I_TELEMETRY_SYMBOLS_PER_BIT_REF;
                    t->secondary = 1;
                    t->secondary_code_length = BEIDOU_B1I_SECONDARY_CODE_LENGTH_REF;
                    t->secondary_code_string = BEIDOU_B1I_SECONDARY_CODE_STR_REF;
                    t->data_secondary_code_length = BEIDOU_B1I_SECONDARY_CODE_LENGTH_REF;
                    t->data_secondary_code_string = BEIDOU_B1I_SECONDARY_CODE_STR_REF;
                }
        }
    memcpy(t->code, code, sizeof(float) * (size_t)code_samples);
    t->code_samples = code_samples;
    t->acq_code_phase_samples = acq_delay_samples;
    t->acq_carrier_doppler_hz = acq_doppler_hz;
    t->acq_sample_stamp = acq_samplestamp;
    t->carrier_doppler_hz = t->acq_carrier_doppler_hz;
    t->carrier_phase_step_rad = TWO_PI_REF * t->carrier_doppler_hz / t->p.fs_in;
    t->carrier_phase_rate_step_rad = 0.0;
    t->hc_n = t->hc_head = t->hk_n = t->hk_head = 0; /* :651-652 */
    for (int k = 0; k < t->n_taps; ++k) t->taps[k] = (tcf){0.0F, 0.0F};
    t->carrier_lock_fail_counter = 0;
    t->code_lock_fail_counter = 0;
    t->rem_code_phase_samples = 0.0;
    t->rem_carr_phase_rad = 0.0F;
    t->rem_code_phase_chips = 0.0;
    t->acc_carrier_phase_rad = 0.0;
    t->cn0_estimation_counter = 0;
    t->carrier_lock_test = 1.0;
    t->CN0_SNV_dB_Hz = 0.0;
    t->EVM = 0.0;
    if (t->veml)
        {
            t->shifts[0] = -t->p.very_early_late_space_chips * (float)t->code_samples_per_chip;
            t->shifts[1] = -t->p.early_late_space_chips * (float)t->code_samples_per_chip;
            t->shifts[2] = 0.0F;
            t->shifts[3] = t->p.early_late_space_chips * (float)t->code_samples_per_chip;
            t->shifts[4] = t->p.very_early_late_space_chips * (float)t->code_samples_per_chip;
        }
    else
        {
            t->shifts[0] = -t->p.early_late_space_chips * (float)t->code_samples_per_chip;
            t->shifts[1] = 0.0F;
            t->shifts[2] = t->p.early_late_space_chips * (float)t->code_samples_per_chip;
        }
    t->prompt_data = (tcf){0.0F, 0.0F};
    t->current_correlation_time_s = t->code_period;
    pll_set_params(&t->carrier_filter, t->p.fll_bw_hz, t->p.pll_bw_hz, t->p.pll_filter_order);
    t->code_filter.bw = t->p.dll_bw_hz;
    lf_update(&t->code_filter);
    t->code_filter.T = (float)t->code_period;
    lf_update(&t->code_filter);
    pll_initialize(&t->carrier_filter, (float)t->acq_carrier_doppler_hz);
    lf_initialize(&t->code_filter, 0.0F);
    t->state = 1;
    t->cloop = 1;
    t->pull_in_transitory = 1;
    t->circ_size = 0;
    t->circ_head = 0;
    t->acc_carrier_phase_initialized = 0;

    /* state 1 (:1813-1844) */
    const int64_t diff = (int64_t)nitems_read - (int64_t)t->acq_sample_stamp;
    const double delta = (double)diff - t->acq_code_phase_samples;
    t->code_freq_chips = t->code_chip_rate;
    t->code_phase_step_chips = t->code_freq_chips / t->p.fs_in;
    t->code_phase_rate_step_chips = 0.0;
    const double T_chip_mod_seconds = 1.0 / t->code_freq_chips;
    const double T_prn_mod_seconds = T_chip_mod_seconds * (double)t->code_length_chips;
    const double T_prn_mod_samples = T_prn_mod_seconds * t->p.fs_in;
    t->acq_code_phase_samples = T_prn_mod_samples - fmod(delta, T_prn_mod_samples);
    t->current_prn_length_samples = (int32_t)round(T_prn_mod_samples);
    const int32_t samples_offset = (int32_t)round(t->acq_code_phase_samples);
    t->acc_carrier_phase_rad -= t->carrier_phase_step_rad * (double)samples_offset;
    t->state = 2;
    sm_reset(&t->cn0_smoother);
    sm_reset(&t->lock_smoother);
    *first_sample = nitems_read + (uint64_t)(int64_t)samples_offset;
    return 0;
}

void orc_trk_stop(orc_trk* t) { t->state = 0; }

/* msg_handler_telemetry_to_trk, tlm_event 1 (:614-637) */
void orc_trk_force_loss_of_lock(orc_trk* t) { t->carrier_lock_fail_counter = 200000; }

/* do_correlation_step (:1064-1089) */
static void do_correlation_step(orc_trk* t, const float* in)
{
    float out[10];
    orc_multicorrelator_real_codes(out, in, t->code, (unsigned)t->code_samples, t->shifts, t->n_taps,
        t->rem_carr_phase_rad, (float)t->carrier_phase_step_rad, (float)t->carrier_phase_rate_step_rad,
        (float)t->rem_code_phase_chips * (float)t->code_samples_per_chip,
        (float)t->code_phase_step_chips * (float)t->code_samples_per_chip,
        (float)t->code_phase_rate_step_chips * (float)t->code_samples_per_chip, t->p.vector_length, t->p.high_dyn, t->assoc);
    for (int k = 0; k < t->n_taps; ++k) t->taps[k] = (tcf){out[2 * k], out[2 * k + 1]};
    if (t->track_pilot)
        {
            /* DATA CORRELATOR (:1078-1088): one tap at the prompt shift on the data code */
            float dout[2];
            orc_multicorrelator_real_codes(dout, in, t->data_code, (unsigned)t->data_code_samples, &t->shifts[t->iP], 1,
                t->rem_carr_phase_rad, (float)t->carrier_phase_step_rad, (float)t->carrier_phase_rate_step_rad,
                (float)t->rem_code_phase_chips * (float)t->code_samples_per_chip,
                (float)t->code_phase_step_chips * (float)t->code_samples_per_chip,
                (float)t->code_phase_rate_step_chips * (float)t->code_samples_per_chip, t->p.vector_length, t->p.high_dyn, t->assoc);
            t->prompt_data = (tcf){dout[0], dout[1]};
        }
}

/* cn0_and_tracking_lock_status (:970-1056) */
static int cn0_and_lock(orc_trk* t, double coh)
{
    const int n = t->p.cn0_samples;
    if (t->cn0_estimation_counter < n)
        {
            t->prompt_buffer[t->cn0_estimation_counter] = t->P_accu;
            t->cn0_estimation_counter++;
            return 1;
        }
    t->prompt_buffer[t->cn0_estimation_counter % n] = t->P_accu;
    t->cn0_estimation_counter++;
    const float cn0_raw = cn0_m2m4(t->prompt_buffer, n, (float)coh);
    t->CN0_SNV_dB_Hz = (double)sm_smooth(&t->cn0_smoother, cn0_raw);
    t->carrier_lock_test = (double)sm_smooth(&t->lock_smoother, carrier_lock_detector(t->prompt_buffer, 1));
    if (!t->pull_in_transitory)
        {
            if (t->carrier_lock_test < t->carrier_lock_threshold)
                t->carrier_lock_fail_counter++;
            else if (t->carrier_lock_fail_counter > 0)
                t->carrier_lock_fail_counter--;
            if (t->CN0_SNV_dB_Hz < t->p.cn0_min)
                t->code_lock_fail_counter++;
            else if (t->code_lock_fail_counter > 0)
                t->code_lock_fail_counter--;
        }
    if (t->carrier_lock_fail_counter > t->p.max_carrier_lock_fail || t->code_lock_fail_counter > t->p.max_code_lock_fail)
        {
            t->carrier_lock_fail_counter = 0;
            t->code_lock_fail_counter = 0;
            return 0;
        }
    /* EVM (:1027-1053) */
    const float I_ref = 1, Q_ref = 0;
    float d, s = 0;
    for (int i = 0; i < n; i++) s = s + t->prompt_buffer[i].re * t->prompt_buffer[i].re;
    d = s / (float)n;
    d = sqrtf(d);
    s = 0;
    for (int i = 0; i < n; i++)
        {
            const float a = fabsf(t->prompt_buffer[i].re / d) - I_ref;
            const float b = fabsf(t->prompt_buffer[i].im / d) - Q_ref;
            s = s + a * a + b * b;
        }
    t->EVM = (double)(s / (float)n / (I_ref * I_ref + Q_ref * Q_ref));
    t->EVM = sqrt(t->EVM);
    return 1;
}

/* run_dll_pll (:1092-1179), enable_doppler_correction = false */
static void run_dll_pll(orc_trk* t)
{
    if (t->cloop)
        t->carr_phase_error_hz = pll_cloop_two_quadrant_atan(t->P_accu) / TWO_PI_REF;
    else
        t->carr_phase_error_hz = pll_four_quadrant_atan(t->P_accu) / TWO_PI_REF;
    if ((t->pull_in_transitory && t->p.enable_fll_pull_in) || t->p.enable_fll_steady_state)
        {
            t->carr_freq_error_hz = fll_diff_atan(t->P_accu_old, t->P_accu, 0, t->current_correlation_time_s) / TWO_PI_REF;
            t->P_accu_old = t->P_accu;
            if (t->pull_in_transitory && t->p.enable_fll_pull_in)
                t->carr_error_filt_hz = (double)pll_get_carrier_error(&t->carrier_filter, (float)t->carr_freq_error_hz,
                    0.0F, (float)t->current_correlation_time_s);
            else
                t->carr_error_filt_hz = (double)pll_get_carrier_error(&t->carrier_filter, (float)t->carr_freq_error_hz,
                    (float)t->carr_phase_error_hz, (float)t->current_correlation_time_s);
        }
    else
        {
            t->carr_error_filt_hz = (double)pll_get_carrier_error(&t->carrier_filter, 0, (float)t->carr_phase_error_hz,
                (float)t->current_correlation_time_s);
        }
    t->carrier_doppler_hz = t->carr_error_filt_hz;
    if (t->veml)
        t->code_error_chips = orc_dll_nc_vemlp_normalized(t->VE_accu, t->E_accu, t->L_accu, t->VL_accu);
    else
        t->code_error_chips = orc_dll_nc_e_minus_l_normalized(t->E_accu.re, t->E_accu.im, t->L_accu.re, t->L_accu.im,
            t->spc, 1.0F, 1.0F);
    t->code_error_filt_chips = (double)lf_apply(&t->code_filter, (float)t->code_error_chips);
    t->code_freq_chips = t->code_chip_rate - t->code_error_filt_chips;
    if (t->p.carrier_aiding) t->code_freq_chips += t->carrier_doppler_hz * t->code_chip_rate / t->signal_carrier_freq;
}

/* boost::circular_buffer::push_back (overwrites the oldest element when full) */
static void hist_push(double* v, double* s, int* n, int* head, int cap, double a, double b)
{
    int slot;
    if (*n < cap)
        {
            slot = (*head + *n) % cap;
            (*n)++;
        }
    else
        {
            slot = *head;
            *head = (*head + 1) % cap;
        }
    v[slot] = a;
    s[slot] = b;
}

/* the rate estimate of :1238-1250 / :1271-1283 */
static double hist_rate(const double* v, const double* s, int head, int cap, int L)
{
    double tmp_cp1 = 0.0, tmp_cp2 = 0.0, tmp_samples = 0.0;
    for (int k = 0; k < L; k++)
        {
            tmp_cp1 += v[(head + k) % cap];
            tmp_cp2 += v[(head + L * 2 - k - 1) % cap];
            tmp_samples += s[(head + L * 2 - k - 1) % cap];
        }
    tmp_cp1 /= (double)L;
    tmp_cp2 /= (double)L;
    return (tmp_cp2 - tmp_cp1) / tmp_samples;
}

/* update_tracking_vars (:1216-1287) */
static void update_tracking_vars(orc_trk* t)
{
    const int L = t->p.smoother_length < 1 ? 1 : (int)t->p.smoother_length; /* dll_pll_conf.cc:119-123 */
    const int cap = 2 * L;
    t->T_chip_seconds = 1.0 / t->code_freq_chips;
    t->T_prn_seconds = t->T_chip_seconds * (double)t->code_length_chips;
    t->T_prn_samples = t->T_prn_seconds * t->p.fs_in;
    t->K_blk_samples = t->T_prn_samples + t->rem_code_phase_samples;
    t->current_prn_length_samples = (int32_t)floor(t->K_blk_samples);
    t->carrier_phase_step_rad = TWO_PI_REF * t->carrier_doppler_hz / t->p.fs_in;
    if (t->p.high_dyn)
        {
            hist_push(t->hc_step, t->hc_samples, &t->hc_n, &t->hc_head, cap, t->carrier_phase_step_rad,
                (double)t->current_prn_length_samples);
            if (t->hc_n == cap) t->carrier_phase_rate_step_rad = hist_rate(t->hc_step, t->hc_samples, t->hc_head, cap, L);
        }
    const double len = (double)t->current_prn_length_samples;
    t->rem_carr_phase_rad += (float)(t->carrier_phase_step_rad * len + 0.5 * t->carrier_phase_rate_step_rad * len * len);
    t->rem_carr_phase_rad = (float)fmod((double)t->rem_carr_phase_rad, TWO_PI_REF);
    t->acc_carrier_phase_rad -= (t->carrier_phase_step_rad * len + 0.5 * t->carrier_phase_rate_step_rad * len * len);
    t->code_phase_step_chips = t->code_freq_chips / t->p.fs_in;
    if (t->p.high_dyn)
        {
            hist_push(t->hk_step, t->hk_samples, &t->hk_n, &t->hk_head, cap, t->code_phase_step_chips,
                (double)t->current_prn_length_samples);
            if (t->hk_n == cap) t->code_phase_rate_step_chips = hist_rate(t->hk_step, t->hk_samples, t->hk_head, cap, L);
        }
    t->rem_code_phase_samples = t->K_blk_samples - len;
    t->rem_code_phase_chips = t->code_freq_chips * t->rem_code_phase_samples / t->p.fs_in;
}

/* acquire_secondary (:923-967) over the preamble circular buffer */
static int acquire_secondary(orc_trk* t)
{
    int32_t corr = 0;
    const int cap = (int)t->secondary_code_length;
    for (int i = 0; i < cap; i++)
        {
            const tcf v = t->circ[(t->circ_head + i) % cap];
            if (v.re < 0.0F)
                corr += (t->secondary_code_string[i] == '0') ? 1 : -1;
            else
                corr += (t->secondary_code_string[i] == '0') ? -1 : 1;
        }
    if (abs(corr) == cap)
        {
            t->flag_pll_180 = corr < 0;
            return 1;
        }
    return 0;
}

static void circ_push(orc_trk* t, tcf v)
{
    const int cap = (int)t->secondary_code_length;
    if (t->circ_size < cap)
        t->circ[(t->circ_head + t->circ_size++) % cap] = v;
    else
        {
            t->circ[t->circ_head] = v;
            t->circ_head = (t->circ_head + 1) % cap;
        }
}

static void fill_output(orc_trk* t, gsdr_trk_epoch* r)
{
    r->prompt_i = (double)t->P_data_accu.re;
    r->prompt_q = (double)t->P_data_accu.im;
    r->flags |= GSDR_TRK_F_VALID_OUTPUT;
}

static int trk_call(orc_trk* t, const float* in, const float* taps_in, uint64_t nitems_read, gsdr_trk_epoch* r);

/* One general_work call (:1784-2152) at input position nitems_read with
 * in = the vector_length input items starting there.  Returns 1 when a record
 * was written (states 2..4), 0 in standby. */
int orc_trk_call(orc_trk* t, const float* in, uint64_t nitems_read, gsdr_trk_epoch* r)
{
    return trk_call(t, in, NULL, nitems_read, r);
}

/* Replay form: the same call with the correlator outputs given (n_taps complex
 * values) instead of computed -- checks the loop restatement of another
 * implementation fed with that implementation's own correlations. */
int orc_trk_call_taps(orc_trk* t, const float* taps, uint64_t nitems_read, gsdr_trk_epoch* r)
{
    return trk_call(t, NULL, taps, nitems_read, r);
}

/* The inputs do_correlation_step passes to the multicorrelator for the channel's
 * next call (:1064-1089), for an external correlator feeding orc_trk_call_taps
 * (the CPU baseline's AVX2 correlator): p[0] rem_carr_phase_rad, p[1]
 * carr_phase_step_rad, p[2] carr_phase_rate_step_rad, p[3] rem_code_phase x spc,
 * p[4] code_phase_step x spc, p[5] code_phase_rate_step x spc; *n_samples =
 * vector_length; *code / *code_samples / shifts[0..n_taps) the replica and taps;
 * returns n_taps. */
int orc_trk_corr_params(const orc_trk* t, float* p, int* n_samples, const float** code, int* code_samples,
    float* shifts)
{
    p[0] = t->rem_carr_phase_rad;
    p[1] = (float)t->carrier_phase_step_rad;
    p[2] = (float)t->carrier_phase_rate_step_rad;
    p[3] = (float)t->rem_code_phase_chips * (float)t->code_samples_per_chip;
    p[4] = (float)t->code_phase_step_chips * (float)t->code_samples_per_chip;
    p[5] = (float)t->code_phase_rate_step_chips * (float)t->code_samples_per_chip;
    *n_samples = (int)t->p.vector_length;
    *code = t->code;
    *code_samples = t->code_samples;
    for (int k = 0; k < t->n_taps; ++k) shifts[k] = t->shifts[k];
    return t->n_taps;
}

/* taps_in: 12 floats -- five complex tap slots (n_taps used) + the data prompt */
static void correlate_or_copy(orc_trk* t, const float* in, const float* taps_in)
{
    if (taps_in)
        {
            for (int k = 0; k < t->n_taps; ++k) t->taps[k] = (tcf){taps_in[2 * k], taps_in[2 * k + 1]};
            if (t->track_pilot) t->prompt_data = (tcf){taps_in[10], taps_in[11]};
        }
    else
        do_correlation_step(t, in);
}

static void cadd(tcf* a, tcf b, float sgn)
{
    if (sgn > 0)
        {
            a->re += b.re;
            a->im += b.im;
        }
    else
        {
            a->re -= b.re;
            a->im -= b.im;
        }
}

/* save_correlation_results (:1288-1400) */
static void save_correlation_results(orc_trk* t)
{
    float sg = 1.0F;
    if (t->secondary)
        {
            sg = t->secondary_code_string[t->current_symbol] == '0' ? 1.0F : -1.0F;
            t->current_symbol++;
            t->current_symbol %= (int32_t)t->secondary_code_length;
        }
    if (t->veml)
        {
            cadd(&t->VE_accu, t->taps[0], sg);
            cadd(&t->VL_accu, t->taps[4], sg);
        }
    cadd(&t->E_accu, t->taps[t->iE], sg);
    cadd(&t->P_accu, t->taps[t->iP], sg);
    cadd(&t->L_accu, t->taps[t->iL], sg);
    const tcf pd = t->track_pilot ? t->prompt_data : t->taps[t->iP];
    if (t->symbols_per_bit > 1)
        {
            if (t->data_secondary_code_length > 0)
                {
                    cadd(&t->P_data_accu, pd, t->data_secondary_code_string[t->current_data_symbol] == '0' ? 1.0F : -1.0F);
                    t->current_data_symbol++;
                    t->current_data_symbol %= (int32_t)t->data_secondary_code_length;
                }
            else
                {
                    cadd(&t->P_data_accu, pd, 1.0F);
                    t->current_data_symbol++;
                    t->current_data_symbol %= t->symbols_per_bit;
                }
        }
    else
        t->P_data_accu = pd;
    t->cloop = t->track_pilot ? 0 : 1;
}

/* log_data (:1403-1500): the dump's accumulator magnitudes, std::abs<float> of the
 * complex accumulators (VE/VL written as 0 without VEML) */
static void log_data(const orc_trk* t, gsdr_trk_epoch* r)
{
    r->flags |= GSDR_TRK_F_LOGGED;
    r->log_accu[0] = t->veml ? hypotf(t->VE_accu.re, t->VE_accu.im) : 0.0F;
    r->log_accu[1] = hypotf(t->E_accu.re, t->E_accu.im);
    r->log_accu[2] = hypotf(t->P_accu.re, t->P_accu.im);
    r->log_accu[3] = hypotf(t->L_accu.re, t->L_accu.im);
    r->log_accu[4] = t->veml ? hypotf(t->VL_accu.re, t->VL_accu.im) : 0.0F;
}

static int trk_call(orc_trk* t, const float* in, const float* taps_in, uint64_t nitems_read, gsdr_trk_epoch* r)
{
    memset(r, 0, sizeof(*r));
    r->sample_counter = nitems_read;
    r->state = t->state;
    int loss_of_lock = 0;
    if (t->pull_in_transitory)
        {
            if ((uint64_t)t->p.pull_in_time_s < (nitems_read - t->acq_sample_stamp) / (uint64_t)(int)t->p.fs_in)
                {
                    t->pull_in_transitory = 0;
                    t->carrier_lock_fail_counter = 0;
                    t->code_lock_fail_counter = 0;
                }
        }
    switch (t->state)
        {
        case 2:
            {
                correlate_or_copy(t, in, taps_in);
                if (t->veml)
                    {
                        t->VE_accu = t->taps[0];
                        t->VL_accu = t->taps[4];
                    }
                t->E_accu = t->taps[t->iE];
                t->P_accu = t->taps[t->iP];
                t->L_accu = t->taps[t->iL];
                t->spc = t->p.early_late_space_chips;
                if ((uint64_t)t->p.bit_synchronization_time_limit_s < (nitems_read - t->acq_sample_stamp) / (uint64_t)(int)t->p.fs_in)
                    t->carrier_lock_fail_counter = 300000;
                if (!cn0_and_lock(t, t->code_period))
                    {
                        clear_tracking_vars(t);
                        t->state = 0;
                        loss_of_lock = 1;
                    }
                else
                    {
                        int next_state = 0;
                        run_dll_pll(t);
                        update_tracking_vars(t);
                        log_data(t, r);
                        if (!t->pull_in_transitory)
                            {
                                if (t->secondary || t->symbols_per_bit > 1)
                                    {
                                        /* secondary code lock / preamble correlation (:1889-1921) */
                                        circ_push(t, t->taps[t->iP]);
                                        if (t->circ_size == (int)t->secondary_code_length) next_state = acquire_secondary(t);
                                    }
                                else
                                    next_state = 1;
                            }
                        if (next_state)
                            {
                                t->VE_accu = t->E_accu = t->P_accu = t->P_data_accu = t->L_accu = t->VL_accu = (tcf){0.0F, 0.0F};
                                t->circ_size = 0;
                                t->circ_head = 0;
                                t->current_symbol = 0;
                                t->current_data_symbol = 0;
                                r->flags |= GSDR_TRK_F_BIT_SYNC;
                                if (t->enable_ext)
                                    {
                                        /* extended correlator: narrow loops and taps (:1945-1983) */
                                        t->extend_count = 0;
                                        t->current_correlation_time_s = (double)((float)t->extend * (float)t->code_period);
                                        t->state = 3;
                                        t->code_filter.T = (float)t->current_correlation_time_s;
                                        lf_update(&t->code_filter);
                                        t->code_filter.bw = t->p.dll_bw_narrow_hz;
                                        lf_update(&t->code_filter);
                                        pll_set_params(&t->carrier_filter, t->p.fll_bw_hz, t->p.pll_bw_narrow_hz, t->p.pll_filter_order);
                                        const float spcf = (float)t->code_samples_per_chip;
                                        if (t->veml)
                                            {
                                                t->shifts[0] = -t->p.very_early_late_space_narrow_chips * spcf;
                                                t->shifts[1] = -t->p.early_late_space_narrow_chips * spcf;
                                                t->shifts[3] = t->p.early_late_space_narrow_chips * spcf;
                                                t->shifts[4] = t->p.very_early_late_space_narrow_chips * spcf;
                                            }
                                        else
                                            {
                                                t->shifts[0] = -t->p.early_late_space_narrow_chips * spcf;
                                                t->shifts[2] = t->p.early_late_space_narrow_chips * spcf;
                                            }
                                        t->spc = t->p.early_late_space_narrow_chips;
                                    }
                                else
                                    t->state = 4;
                            }
                    }
                break;
            }
        case 3:
            {
                /* coherent integration (:1989-2026) */
                correlate_or_copy(t, in, taps_in);
                save_correlation_results(t);
                update_tracking_vars(t);
                if (t->current_data_symbol == 0)
                    {
                        log_data(t, r);
                        fill_output(t, r);
                        t->P_data_accu = (tcf){0.0F, 0.0F};
                    }
                t->extend_count++;
                if (t->extend_count == t->extend - 1)
                    {
                        t->extend_count = 0;
                        t->state = 4;
                    }
                break;
            }
        case 4:
            {
                correlate_or_copy(t, in, taps_in);
                save_correlation_results(t);
                if (!cn0_and_lock(t, t->code_period * (double)t->extend))
                    {
                        clear_tracking_vars(t);
                        t->state = 0;
                        loss_of_lock = 1;
                    }
                else
                    {
                        run_dll_pll(t);
                        update_tracking_vars(t);
                        if (!t->acc_carrier_phase_initialized)
                            {
                                t->acc_carrier_phase_rad = -(double)t->rem_carr_phase_rad;
                                t->acc_carrier_phase_initialized = 1;
                            }
                        if (t->current_data_symbol == 0)
                            {
                                log_data(t, r);
                                fill_output(t, r);
                                t->P_data_accu = (tcf){0.0F, 0.0F};
                            }
                        t->VE_accu = t->E_accu = t->P_accu = t->L_accu = t->VL_accu = (tcf){0.0F, 0.0F};
                        if (t->enable_ext) t->state = 3;
                    }
                break;
            }
        default:
            return 0;
        }
    for (int k = 0; k < t->n_taps; ++k)
        {
            r->taps[2 * k] = t->taps[k].re;
            r->taps[2 * k + 1] = t->taps[k].im;
        }
    r->data_prompt[0] = t->prompt_data.re;
    r->data_prompt[1] = t->prompt_data.im;
    r->carrier_rate = (float)t->carrier_phase_rate_step_rad;
    r->code_rate = (float)t->code_phase_rate_step_chips;
    r->carr_phase_error_hz = (float)t->carr_phase_error_hz;
    r->carr_error_filt_hz = (float)t->carr_error_filt_hz;
    r->code_error_chips = (float)t->code_error_chips;
    r->code_error_filt_chips = (float)t->code_error_filt_chips;
    if (loss_of_lock) r->flags |= GSDR_TRK_F_LOSS_OF_LOCK;
    if (t->flag_pll_180) r->flags |= GSDR_TRK_F_PLL_180;
    r->consumed = t->current_prn_length_samples;
    r->rem_carr_phase_rad = t->rem_carr_phase_rad;
    r->carrier_doppler_hz = t->carrier_doppler_hz;
    r->code_freq_chips = t->code_freq_chips;
    r->rem_code_phase_samples = t->rem_code_phase_samples;
    r->acc_carrier_phase_rad = t->acc_carrier_phase_rad;
    r->cn0_db_hz = t->CN0_SNV_dB_Hz;
    r->carrier_lock_test = t->carrier_lock_test;
    r->evm = t->EVM;
    return 1;
}

int32_t orc_trk_state(const orc_trk* t) { return t->state; }
int32_t orc_trk_vector_length(const orc_trk* t) { return (int32_t)t->p.vector_length; }

/* Loop-filter probe for the reference's tracking_loop_filter_test.cc vectors. */
void orc_loop_filter_run(int order, int last_int, float bw, float T, const float* in, float* out, int n)
{
    lf_t f;
    lf_init(&f, T, bw, order, last_int);
    lf_initialize(&f, 0.0F);
    for (int i = 0; i < n; ++i) out[i] = lf_apply(&f, in[i]);
}
