/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the VOLK-GNSSSDR protokernels that sit on the tracking and
 * acquisition hot path of GNSS-SDR.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker /
 * CPU baseline.  The product path (gnss-sdr-new_amd/) never links it.
 *
 * Parity status: the reference's own VOLK sources cannot be built here (their
 * public header volk_gnsssdr/volk_gnsssdr.h is Mako-generated code), so this file
 * restates the *generic* protokernels from their published arithmetic.  It is
 * pinned indirectly: the acquisition chain that uses these semantics reproduces
 * the reference's golden results on the reference's own IQ captures
 * (tests/test_oracle_golden.py), and the known-answer tables of IS-GPS-200 pin
 * the code generator.  Kernel-level values are otherwise "parity unpinned".
 *
 * Every function cites the reference file:line it restates.  Paths are relative
 * to the reference root; KERN/ = src/algorithms/libs/volk_gnsssdr_module/
 * volk_gnsssdr/kernels/volk_gnsssdr/volk_gnsssdr_.
 *
 * Build: cc -O2 -ffp-contract=off -fno-fast-math -fPIC -shared (oracle/Makefile).
 * -ffp-contract=off matters: the generic kernels are plain C without FMA.
 */
#include <complex.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef struct { float re, im; } cf32;

static inline cf32 cmul(cf32 a, cf32 b)
{
    /* C99 complex float product as gcc evaluates it for finite operands:
     * (ac - bd) + i(ad + bc), no contraction. */
    cf32 r;
    float ac = a.re * b.re, bd = a.im * b.im, ad = a.re * b.im, bc = a.im * b.re;
    r.re = ac - bd;
    r.im = ad + bc;
    return r;
}

static inline cf32 cscale(cf32 a, float s)
{
    cf32 r = {a.re * s, a.im * s};
    return r;
}

/* ------------------------------------------------------------------------ */
/* Code-phase index with the two float associations found in the reference.  */
/* assoc 0: KERN/32f_xn_resampler_32f_xn.h:73   floor((step*n + shift) - rem) */
/* assoc 1: KERN/32f_xn_resampler_32f_xn.h:384-390 (a_avx, x86 dispatch)      */
/*          floor(step*n + (shift - rem)), n built as float lane counters.     */
/* Both wrap negatives by whole code periods then take the modulo (:75-76).    */
/* ------------------------------------------------------------------------ */
static inline int wrap_index(int idx, unsigned int L)
{
    if (idx < 0) idx += (int)L * (abs(idx) / (int)L + 1);
    return idx % (int)L;
}

static inline int code_index(float step, float shift, float rem, unsigned int n, unsigned int L, int assoc)
{
    float t;
    if (assoc == 0)
        {
            volatile float a = step * (float)n;
            volatile float b = a + shift;
            t = b - rem;
        }
    else
        {
            volatile float a = step * (float)n;
            volatile float b = shift - rem;
            t = a + b;
        }
    return wrap_index((int)floorf(t), L);
}

/* KERN/32f_xn_resampler_32f_xn.h:63-80 (generic) and :362-438 (a_avx association).
 * out is K rows of N floats, row-major. */
void orc_resampler_32f_xn(float* out, const float* code, float rem, float step,
    const float* shifts, unsigned int L, int K, unsigned int N, int assoc)
{
    for (int k = 0; k < K; k++)
        for (unsigned int n = 0; n < N; n++)
            out[(size_t)k * N + n] = code[code_index(step, shifts[k], rem, n, L, assoc)];
}

/* Same index arithmetic, returning the indices (for bit-exact checks). */
void orc_resampler_index(int32_t* out, float rem, float step, const float* shifts,
    unsigned int L, int K, unsigned int N, int assoc)
{
    for (int k = 0; k < K; k++)
        for (unsigned int n = 0; n < N; n++)
            out[(size_t)k * N + n] = code_index(step, shifts[k], rem, n, L, assoc);
}

/* KERN/32fc_xn_resampler_32fc_xn.h:60-82 (complex code replicas, generic). */
void orc_resampler_32fc_xn(float* out, const float* code, float rem, float step,
    const float* shifts, unsigned int L, int K, unsigned int N, int assoc)
{
    const cf32* c = (const cf32*)code;
    cf32* o = (cf32*)out;
    for (int k = 0; k < K; k++)
        for (unsigned int n = 0; n < N; n++)
            o[(size_t)k * N + n] = c[code_index(step, shifts[k], rem, n, L, assoc)];
}

/* KERN/32f_xn_high_dynamics_resampler_32f_xn.h:67-96 (generic).
 * Tap 0 carries the code-rate term; taps 1..K-1 are circularly sample-shifted
 * copies of tap 0 by round(delta_shift / step) samples (cumulative). */
void orc_high_dyn_resampler_32f_xn(float* out, const float* code, float rem, float step,
    float rate, const float* shifts, unsigned int L, int K, unsigned int N)
{
    for (unsigned int n = 0; n < N; n++)
        {
            volatile float a = step * (float)n;
            volatile float b = rate * (float)(n * n);
            volatile float c = a + b;
            volatile float d = c + shifts[0];
            float t = d - rem;
            out[n] = code[wrap_index((int)floor(t), L)];
        }
    unsigned int sh = 0;
    for (int k = 1; k < K; k++)
        {
            sh += (int)round((shifts[k] - shifts[k - 1]) / step);
            memcpy(&out[(size_t)k * N], &out[sh], (N - sh) * sizeof(float));
            memcpy(&out[(size_t)k * N + (N - sh)], &out[0], sh * sizeof(float));
        }
}

/* KERN/32fc_32f_rotator_dot_prod_32fc_xn.h:66-98 (generic).
 * res[k] = sum_n (x[n] * ph_n) * a_k[n]; phase is renormalised when n % 256 == 0
 * (after ph_n has been used), then advanced by phase_inc.  phase is in/out. */
void orc_rotator_dot_prod_32fc_32f_xn(float* result, const float* in, float inc_re, float inc_im,
    float* phase, const float* a, int K, unsigned int N)
{
    cf32* res = (cf32*)result;
    const cf32* x = (const cf32*)in;
    cf32 inc = {inc_re, inc_im};
    cf32 ph = {phase[0], phase[1]};
    for (int k = 0; k < K; k++) res[k].re = res[k].im = 0.0f;
    for (unsigned int n = 0; n < N; n++)
        {
            cf32 t = cmul(x[n], ph);
            if (n % 256 == 0)
                {
                    float m = hypotf(ph.re, ph.im);
                    ph.re /= m;
                    ph.im /= m;
                }
            ph = cmul(ph, inc);
            for (int k = 0; k < K; k++)
                {
                    cf32 p = cscale(t, a[(size_t)k * N + n]);
                    res[k].re += p.re;
                    res[k].im += p.im;
                }
        }
    phase[0] = ph.re;
    phase[1] = ph.im;
}

/* KERN/32fc_32f_rotator_dot_prod_32fc_xn.h:155-314 (u_avx) and :318-480 (a_avx,
 * identical arithmetic): the kernel the reference's dispatcher runs on x86 with AVX
 * (VOLK/lib/volk_gnsssdr_rank_archs.c:76-100 picks the highest-ranked machine).
 * Sixteen phasor lanes z_j = phase * inc^j (C complex products, :188-193), each
 * advanced by dz = inc^16 (four squarings, :200-204; normalised once, :211)
 * after it is used; lane j of block m accumulates (x[16m+j] z_j) a_k[16m+j] in its
 * own accumulator (:222-253); the lanes are renormalised when m % 64 == 0, after
 * the block's update (:257-263); the 16 accumulators are summed as
 * ((v_j + v_{4+j}) + v_{8+j}) + v_{12+j} per j < 4, then 0 + s_0 + s_1 + s_2 + s_3
 * (:266-279); the tail continues from lane 0's phasor, normalised (:282-296), with
 * the scalar product order of the generic kernel.
 * _mm256_complexmul_ps (volk_gnsssdr_avx_intrinsics.h:20-29) = cmul;
 * _mm256_complexnormalise_ps (:56-63): z / sqrtf(re*re + im*im) by division. */
static inline cf32 cnorm_avx(cf32 z)
{
    const float r = sqrtf(z.re * z.re + z.im * z.im);
    cf32 o = {z.re / r, z.im / r};
    return o;
}

void orc_rotator_dot_prod_32fc_32f_xn_avx(float* result, const float* in, float inc_re, float inc_im,
    float* phase, const float* a, int K, unsigned int N)
{
    cf32* res = (cf32*)result;
    const cf32* x = (const cf32*)in;
    const cf32 inc = {inc_re, inc_im};
    cf32 ph = {phase[0], phase[1]};
    const unsigned int sixteenth = N / 16;
    cf32 z[16];
    for (int j = 0; j < 16; j++)
        {
            z[j] = ph;
            ph = cmul(ph, inc);
        }
    cf32 dz = inc;
    dz = cmul(dz, dz);
    dz = cmul(dz, dz);
    dz = cmul(dz, dz);
    dz = cmul(dz, dz);
    dz = cnorm_avx(dz);
    cf32* acc = (cf32*)calloc((size_t)K * 16, sizeof(cf32));
    for (unsigned int m = 0; m < sixteenth; m++)
        {
            cf32 t[16];
            for (int j = 0; j < 16; j++)
                {
                    t[j] = cmul(x[16 * m + j], z[j]);
                    z[j] = cmul(z[j], dz);
                }
            for (int k = 0; k < K; k++)
                for (int j = 0; j < 16; j++)
                    {
                        const float b = a[(size_t)k * N + 16 * m + j];
                        cf32* v = &acc[(size_t)k * 16 + j];
                        const float cr = t[j].re * b, ci = t[j].im * b;
                        v->re = cr + v->re;
                        v->im = ci + v->im;
                    }
            if (m % 64 == 0)
                for (int j = 0; j < 16; j++) z[j] = cnorm_avx(z[j]);
        }
    for (int k = 0; k < K; k++)
        {
            const cf32* v = &acc[(size_t)k * 16];
            cf32 r = {0.0f, 0.0f};
            for (int j = 0; j < 4; j++)
                {
                    cf32 s;
                    s.re = ((v[j].re + v[4 + j].re) + v[8 + j].re) + v[12 + j].re;
                    s.im = ((v[j].im + v[4 + j].im) + v[8 + j].im) + v[12 + j].im;
                    r.re += s.re;
                    r.im += s.im;
                }
            res[k] = r;
        }
    free(acc);
    ph = cnorm_avx(z[0]);
    for (unsigned int n = sixteenth * 16; n < N; n++)
        {
            const cf32 wo = cmul(x[n], ph);
            ph = cmul(ph, inc);
            for (int k = 0; k < K; k++)
                {
                    const cf32 p = cscale(wo, a[(size_t)k * N + n]);
                    res[k].re += p.re;
                    res[k].im += p.im;
                }
        }
    phase[0] = ph.re;
    phase[1] = ph.im;
}

/* KERN/32fc_x2_rotator_dot_prod_32fc_xn.h:67-104 (generic, complex replicas). */
void orc_rotator_dot_prod_32fc_x2_xn(float* result, const float* in, float inc_re, float inc_im,
    float* phase, const float* a, int K, unsigned int N)
{
    cf32* res = (cf32*)result;
    const cf32* x = (const cf32*)in;
    const cf32* ac = (const cf32*)a;
    cf32 inc = {inc_re, inc_im};
    cf32 ph = {phase[0], phase[1]};
    for (int k = 0; k < K; k++) res[k].re = res[k].im = 0.0f;
    for (unsigned int n = 0; n < N; n++)
        {
            cf32 t = cmul(x[n], ph);
            if (n % 256 == 0)
                {
                    float m = hypotf(ph.re, ph.im);
                    ph.re /= m;
                    ph.im /= m;
                }
            ph = cmul(ph, inc);
            for (int k = 0; k < K; k++)
                {
                    cf32 p = cmul(t, ac[(size_t)k * N + n]);
                    res[k].re += p.re;
                    res[k].im += p.im;
                }
        }
    phase[0] = ph.re;
    phase[1] = ph.im;
}

/* KERN/32fc_32f_high_dynamic_rotator_dot_prod_32fc_xn.h:68-112 (generic, glibc path).
 * Sample n is rotated by the phase left by iteration n-1:
 * ph_0 = phase; ph_n = phase * inc^n * rate^((n-1)^2) (renormalised) for n >= 1. */
void orc_high_dyn_rotator_dot_prod_32fc_32f_xn(float* result, const float* in, float inc_re, float inc_im,
    float rate_re, float rate_im, float* phase, const float* a, int K, unsigned int N)
{
    cf32* res = (cf32*)result;
    const cf32* x = (const cf32*)in;
    cf32 inc = {inc_re, inc_im};
    float complex rate = rate_re + I * rate_im;
    cf32 ph = {phase[0], phase[1]};
    cf32 ph_dop = ph;
    for (int k = 0; k < K; k++) res[k].re = res[k].im = 0.0f;
    for (unsigned int n = 0; n < N; n++)
        {
            if (n % 256 == 0)
                {
                    float m = hypotf(ph.re, ph.im);
                    ph.re /= m;
                    ph.im /= m;
                }
            cf32 t = cmul(x[n], ph);
            ph_dop = cmul(ph_dop, inc);
            float complex r = cpowf(rate, (float)(n * n) + I * 0.0f);
            float m = hypotf(crealf(r), cimagf(r));
            cf32 pr = {crealf(r) / m, cimagf(r) / m};
            ph = cmul(ph_dop, pr);
            for (int k = 0; k < K; k++)
                {
                    cf32 p = cscale(t, a[(size_t)k * N + n]);
                    res[k].re += p.re;
                    res[k].im += p.im;
                }
        }
    phase[0] = ph.re;
    phase[1] = ph.im;
}

/* KERN/s32f_sincos_32fc.h:390-403 (generic): fp32-accumulated phase, cosf/sinf. */
void orc_s32f_sincos_32fc(float* out, float phase_inc, float* phase, unsigned int N)
{
    float p = *phase;
    for (unsigned int i = 0; i < N; i++)
        {
            out[2 * i] = cosf(p);
            out[2 * i + 1] = sinf(p);
            p += phase_inc;
        }
    *phase = p;
}

/* KERN/s32f_sincos_32fc.h:448-627 (a_avx2 / u_avx2, the kernel the reference's
 * dispatcher picks on an AVX2 x86-64 host): eight lanes start at phase + k*inc and
 * advance by 8*inc (fp32), each lane's cos/sin from the Cephes polynomials after
 * the three-constant range reduction; the N % 8 tail continues from
 * phase + inc * (8 * iters) with cosf/sinf.  Restated per lane in the same fp32
 * operation order (the file is built with -ffp-contract=off). */
static void cephes_sincos_f32(float x0, float* s, float* c)
{
    const float FOPI = 1.27323954473516f;
    const float DP1 = -0.78515625f, DP2 = -2.4187564849853515625e-4f, DP3 = -3.77489497744594108e-8f;
    const float C0 = 2.443315711809948E-005f, C1 = -1.388731625493765E-003f, C2 = 4.166664568298827E-002f;
    const float S0 = -1.9515295891E-4f, S1 = 8.3321608736E-3f, S2 = -1.6666654611E-1f;
    int sign_sin = signbit(x0) ? 1 : 0;
    float x = fabsf(x0);
    float y = x * FOPI;
    int32_t j = (int32_t)y; /* cvttps: truncation (|y| < 2^31 here) */
    j = (j + 1) & ~1;
    y = (float)j;
    const int swap = (j & 4) != 0;
    const int poly = (j & 2) == 0;
    x = x + y * DP1;
    x = x + y * DP2;
    x = x + y * DP3;
    const int sign_cos = ((~(j - 2)) & 4) != 0;
    sign_sin ^= swap;
    const float z = x * x;
    float yc = C0 * z;
    yc = yc + C1;
    yc = yc * z;
    yc = yc + C2;
    yc = yc * z;
    yc = yc * z;
    yc = yc - z * 0.5f;
    yc = yc + 1.0f;
    float ys = S0 * z;
    ys = ys + S1;
    ys = ys * z;
    ys = ys + S2;
    ys = ys * z;
    ys = ys * x;
    ys = ys + x;
    float sv = poly ? ys : yc, cv = poly ? yc : ys;
    *s = sign_sin ? -sv : sv;
    *c = sign_cos ? -cv : cv;
}

void orc_s32f_sincos_32fc_avx2(float* out, float phase_inc, float* phase, unsigned int N)
{
    const float p0 = *phase;
    const unsigned int iters = N / 8;
    float lane[8];
    for (int k = 0; k < 8; k++) lane[k] = k == 0 ? p0 : p0 + (float)k * phase_inc;
    const float inc8 = 8.0f * phase_inc;
    for (unsigned int it = 0; it < iters; it++)
        for (int k = 0; k < 8; k++)
            {
                cephes_sincos_f32(lane[k], &out[2 * (8 * it + k) + 1], &out[2 * (8 * it + k)]);
                lane[k] = lane[k] + inc8;
            }
    float p = p0 + phase_inc * (float)(iters * 8);
    for (unsigned int i = iters * 8; i < N; i++)
        {
            out[2 * i] = cosf(p);
            out[2 * i + 1] = sinf(p);
            p += phase_inc;
        }
    *phase = p;
}

/* KERN/32f_index_max_32u.h:446-467 (generic): first index of the maximum (strict >). */
uint32_t orc_index_max_32u(const float* src, uint32_t N)
{
    if (N == 0) return 0;
    float m = src[0];
    uint32_t idx = 0;
    for (uint32_t i = 1; i < N; i++)
        if (src[i] > m)
            {
                m = src[i];
                idx = i;
            }
    return idx;
}

/* ------------------------------------------------------------------------ */
/* Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler  */
/* src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.cc:103-126:    */
/* update_local_code (:75-100) then the rotator dot product with               */
/* phase_offset = (cos rem, -sin rem) and phase_inc = exp(-j step) in float.   */
/* ------------------------------------------------------------------------ */
void orc_multicorrelator_real_codes(float* out, const float* sig, const float* code, unsigned int L,
    const float* shifts, int K, float rem_carr, float carr_step, float carr_rate,
    float rem_code, float code_step, float code_rate, unsigned int N, int high_dyn, int assoc)
{
    float* rs = (float*)malloc((size_t)K * N * sizeof(float));
    if (high_dyn)
        orc_high_dyn_resampler_32f_xn(rs, code, rem_code, code_step, code_rate, shifts, L, K, N);
    else
        orc_resampler_32f_xn(rs, code, rem_code, code_step, shifts, L, K, N, assoc);
    float ph[2] = {cosf(rem_carr), -sinf(rem_carr)};
    float complex inc = cexpf(0.0f + I * (-carr_step));
    if (high_dyn)
        {
            float complex rate = cexpf(0.0f + I * (-carr_rate));
            orc_high_dyn_rotator_dot_prod_32fc_32f_xn(out, sig, crealf(inc), cimagf(inc),
                crealf(rate), cimagf(rate), ph, rs, K, N);
        }
    else
        {
            orc_rotator_dot_prod_32fc_32f_xn(out, sig, crealf(inc), cimagf(inc), ph, rs, K, N);
        }
    free(rs);
}

/* The same correlator call with the rotator the reference dispatches on x86
 * (u_avx / a_avx above) after the a_avx resampler association (assoc 1). */
void orc_multicorrelator_real_codes_avx(float* out, const float* sig, const float* code, unsigned int L,
    const float* shifts, int K, float rem_carr, float carr_step, float rem_code, float code_step, unsigned int N)
{
    float* rs = (float*)malloc((size_t)K * N * sizeof(float));
    orc_resampler_32f_xn(rs, code, rem_code, code_step, shifts, L, K, N, 1);
    float ph[2] = {cosf(rem_carr), -sinf(rem_carr)};
    float complex inc = cexpf(0.0f + I * (-carr_step));
    orc_rotator_dot_prod_32fc_32f_xn_avx(out, sig, crealf(inc), cimagf(inc), ph, rs, K, N);
    free(rs);
}

/* Cpu_Multicorrelator::Carrier_wipeoff_multicorrelator_resampler
 * src/algorithms/tracking/libs/cpu_multicorrelator.cc:73-100 (complex codes). */
void orc_multicorrelator_complex_codes(float* out, const float* sig, const float* code, unsigned int L,
    const float* shifts, int K, float rem_carr, float carr_step, float rem_code, float code_step,
    unsigned int N, int assoc)
{
    float* rs = (float*)malloc((size_t)K * N * 2 * sizeof(float));
    orc_resampler_32fc_xn(rs, code, rem_code, code_step, shifts, L, K, N, assoc);
    float ph[2] = {cosf(rem_carr), -sinf(rem_carr)};
    float complex inc = cexpf(0.0f + I * (-carr_step));
    orc_rotator_dot_prod_32fc_x2_xn(out, sig, crealf(inc), cimagf(inc), ph, rs, K, N);
    free(rs);
}

/* "Exact" companion: the same phase model as the reference (the float-rounded
 * phase_offset and phase_inc define the rotation angles) evaluated with a
 * unit-modulus phasor in double precision and fp64 accumulation.  This is the
 * value both the reference and the GPU approximate; used to measure how close
 * each one is. */
void orc_multicorrelator_real_codes_exact(double* out, const float* sig, const float* code, unsigned int L,
    const float* shifts, int K, float rem_carr, float carr_step, float rem_code, float code_step,
    unsigned int N, int assoc)
{
    float complex inc = cexpf(0.0f + I * (-carr_step));
    double th = atan2((double)cimagf(inc), (double)crealf(inc));
    double ps = atan2((double)(-sinf(rem_carr)), (double)cosf(rem_carr));
    for (int k = 0; k < 2 * K; k++) out[k] = 0.0;
    for (unsigned int n = 0; n < N; n++)
        {
            double phi = ps + th * (double)n;
            double c = cos(phi), s = sin(phi);
            double xr = sig[2 * n], xi = sig[2 * n + 1];
            double tr = xr * c - xi * s, ti = xr * s + xi * c;
            for (int k = 0; k < K; k++)
                {
                    double a = code[code_index(code_step, shifts[k], rem_code, n, L, assoc)];
                    out[2 * k] += tr * a;
                    out[2 * k + 1] += ti * a;
                }
        }
}
