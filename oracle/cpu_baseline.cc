// ORACLE / CPU BASELINE -- measurement and test infrastructure only: bench.py's
// cpu_baseline leg and tests/ load it, the product path never does.
//
// A multi-threaded C++ restatement of the reference's CPU path for the bench
// workload, timed on the GPU box's host cores:
//
//  * pcps_acquisition::acquisition_core for a batch of PRNs on one block
//    (src/algorithms/acquisition/gnuradio_blocks/pcps_acquisition.cc:655-696):
//    per Doppler bin d, X_d = FFT(x .* w_d) (:658-662), then per PRN
//    |IFFT(X_d .* conj(C_p))|^2 (:664-674) reduced to the row maximum, its first
//    index and the row sum, and max_to_input_power_statistic (:511-543) over the
//    rows.  The wipe-off rows accumulate their phase in fp32 like the generic
//    volk_gnsssdr_s32f_sincos_32fc (KERN/s32f_sincos_32fc.h:390-403).
//    FFT: this file's own mixed-radix (2,3,4,5) Stockham transform, 8 transforms
//    per AVX2 vector (8 PRNs, or 8 Doppler rows, in the SIMD lanes).  The image has
//    neither FFTW3f nor a pocketfft header; the report says so.
//  * dll_pll_veml_tracking's correlation step (:1064-1089):
//    Cpu_Multicorrelator_Real_Codes -> volk_gnsssdr_32f_xn_resampler_32f_xn +
//    volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn, fused here in one AVX2 pass
//    (code index in the AVX protokernel's association
//    floor(step*n + (shift - rem)), KERN/32f_xn_resampler_32f_xn.h:384-390; a
//    rotating phasor renormalised every 256 samples), feeding the oracle's loop
//    restatement (trk_oracle.c, orc_trk_call_taps) for the DLL/PLL update.
//  * std::thread over (Doppler bin, PRN group) tasks and over channels.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <complex>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>
#include <vector>

#include "../include/gsdr.h"

extern "C" {
typedef struct orc_trk orc_trk;
int orc_trk_corr_params(const orc_trk* t, float* p, int* n_samples, const float** code, int* code_samples,
    float* shifts);
int orc_trk_call_taps(orc_trk* t, const float* taps, uint64_t nitems_read, gsdr_trk_epoch* r);
int orc_trk_call(orc_trk* t, const float* in, uint64_t nitems_read, gsdr_trk_epoch* r);
}

namespace
{
typedef float v8 __attribute__((vector_size(32)));
typedef int32_t v8i __attribute__((vector_size(32)));

struct cv
{
    v8 r, i;
};

inline v8 bc(float x) { return v8{x, x, x, x, x, x, x, x}; }
inline cv add(cv a, cv b) { return {a.r + b.r, a.i + b.i}; }
inline cv sub(cv a, cv b) { return {a.r - b.r, a.i - b.i}; }
inline cv mul_mi(cv a) { return {a.i, -a.r}; }  // (-i) a
inline cv cmul(cv a, float wr, float wi) { return {a.r * wr - a.i * wi, a.r * wi + a.i * wr}; }
inline cv scale(cv a, float s) { return {a.r * s, a.i * s}; }

// ---- small forward DFTs, exp(-2 pi i nk / R), in place
inline void dft2(cv* v)
{
    const cv a = v[0], b = v[1];
    v[0] = add(a, b);
    v[1] = sub(a, b);
}
inline void dft3(cv* v)
{
    const float h = 0.86602540378443864676f;
    const cv s = add(v[1], v[2]), d = sub(v[1], v[2]);
    const cv m = {v[0].r - 0.5f * s.r, v[0].i - 0.5f * s.i};
    const cv t = scale(mul_mi(d), h);
    v[0] = add(v[0], s);
    v[1] = add(m, t);
    v[2] = sub(m, t);
}
inline void dft4(cv* v)
{
    const cv a = add(v[0], v[2]), b = sub(v[0], v[2]);
    const cv c = add(v[1], v[3]), d = mul_mi(sub(v[1], v[3]));
    v[0] = add(a, c);
    v[2] = sub(a, c);
    v[1] = add(b, d);
    v[3] = sub(b, d);
}
inline void dft5(cv* v)
{
    const float c1 = 0.30901699437494742410f, c2 = -0.80901699437494742410f;
    const float s1 = 0.95105651629515357212f, s2 = 0.58778525229247312917f;
    const cv a1 = add(v[1], v[4]), b1 = sub(v[1], v[4]);
    const cv a2 = add(v[2], v[3]), b2 = sub(v[2], v[3]);
    const cv x0 = v[0];
    const cv p1 = {x0.r + c1 * a1.r + c2 * a2.r, x0.i + c1 * a1.i + c2 * a2.i};
    const cv p2 = {x0.r + c2 * a1.r + c1 * a2.r, x0.i + c2 * a1.i + c1 * a2.i};
    const cv q1 = mul_mi({s1 * b1.r + s2 * b2.r, s1 * b1.i + s2 * b2.i});
    const cv q2 = mul_mi({s2 * b1.r - s1 * b2.r, s2 * b1.i - s1 * b2.i});
    v[0] = add(x0, add(a1, a2));
    v[1] = add(p1, q1);
    v[4] = sub(p1, q1);
    v[2] = add(p2, q2);
    v[3] = sub(p2, q2);
}

inline void dft8(cv* v)
{
    // 2 x 4: radix-4 DFTs of the even and odd halves, W8 twiddles, radix-2 combine
    const float h = 0.70710678118654752440f;
    cv e[4] = {v[0], v[2], v[4], v[6]}, o[4] = {v[1], v[3], v[5], v[7]};
    dft4(e);
    dft4(o);
    // o[k] *= W8^k: W8 = (h, -h), W8^2 = -i, W8^3 = (-h, -h)
    o[1] = {(o[1].r + o[1].i) * h, (o[1].i - o[1].r) * h};
    o[2] = mul_mi(o[2]);
    o[3] = {(o[3].i - o[3].r) * h, -(o[3].r + o[3].i) * h};
    for (int k = 0; k < 4; ++k)
        {
            v[k] = add(e[k], o[k]);
            v[k + 4] = sub(e[k], o[k]);
        }
}

template <int R>
inline void dft(cv* v)
{
    if constexpr (R == 2)
        dft2(v);
    else if constexpr (R == 3)
        dft3(v);
    else if constexpr (R == 4)
        dft4(v);
    else if constexpr (R == 5)
        dft5(v);
    else
        dft8(v);
}

// One Stockham stage: butterfly j = q*Ns + k reads x[j + r*m], twiddles by
// W_{Ns R}^{r k}, writes y[q*Ns*R + k + r*Ns].
template <int R>
void stage(const cv* __restrict x, cv* __restrict y, const float* __restrict tw, int n, int Ns)
{
    const int m = n / R;
    for (int q = 0; q < m / Ns; ++q)
        {
            {
                // k = 0: no twiddle
                const int j = q * Ns;
                cv v[R];
                for (int r = 0; r < R; ++r) v[r] = x[j + r * m];
                dft<R>(v);
                cv* o = y + static_cast<size_t>(q) * Ns * R;
                for (int r = 0; r < R; ++r) o[r * Ns] = v[r];
            }
            for (int k = 1; k < Ns; ++k)
                {
                    const int j = q * Ns + k;
                    cv v[R];
                    for (int r = 0; r < R; ++r) v[r] = x[j + r * m];
                    const float* w = tw + static_cast<size_t>(k) * (R - 1) * 2;
                    for (int r = 1; r < R; ++r) v[r] = cmul(v[r], w[2 * (r - 1)], w[2 * (r - 1) + 1]);
                    dft<R>(v);
                    cv* o = y + static_cast<size_t>(q) * Ns * R + k;
                    for (int r = 0; r < R; ++r) o[r * Ns] = v[r];
                }
        }
}

// ---- batched Stockham FFT plan: N = prod(radix), 8 transforms per vector
struct Plan
{
    int n{0};
    std::vector<int> radix;
    std::vector<std::vector<float>> tw;  // per stage: Ns x (R-1) complex, interleaved
    bool make(int N)
    {
        n = N;
        radix.clear();
        int m = N;
        for (int r : {8, 4, 2, 3, 5})
            while (m % r == 0)
                {
                    radix.push_back(r);
                    m /= r;
                }
        if (m != 1) return false;
        tw.clear();
        int Ns = 1;
        for (int R : radix)
            {
                std::vector<float> t(static_cast<size_t>(Ns) * (R - 1) * 2);
                for (int k = 0; k < Ns; ++k)
                    for (int r = 1; r < R; ++r)
                        {
                            const double a = -2.0 * M_PI * (double)(r * k) / (double)(Ns * R);
                            t[(static_cast<size_t>(k) * (R - 1) + (r - 1)) * 2] = (float)std::cos(a);
                            t[(static_cast<size_t>(k) * (R - 1) + (r - 1)) * 2 + 1] = (float)std::sin(a);
                        }
                tw.push_back(std::move(t));
                Ns *= R;
            }
        return true;
    }
    // forward transform of 8 interleaved sequences: src -> (ping-pong) -> result
    // pointer (src or tmp)
    cv* run(cv* src, cv* tmp) const
    {
        cv* x = src;
        cv* y = tmp;
        int Ns = 1;
        for (size_t s = 0; s < radix.size(); ++s)
            {
                const int R = radix[s];
                const float* t = tw[s].data();
                switch (R)
                    {
                    case 2: stage<2>(x, y, t, n, Ns); break;
                    case 3: stage<3>(x, y, t, n, Ns); break;
                    case 4: stage<4>(x, y, t, n, Ns); break;
                    case 5: stage<5>(x, y, t, n, Ns); break;
                    default: stage<8>(x, y, t, n, Ns); break;
                    }
                std::swap(x, y);
                Ns *= R;
            }
        return x;
    }
};

struct RowStat
{
    float max;
    uint32_t idx;
    float sum;
};

void* aligned_alloc64(size_t bytes)
{
    void* p = nullptr;
    if (posix_memalign(&p, 64, (bytes + 63) / 64 * 64) != 0) return nullptr;
    return p;
}

template <class F>
void parallel(int nthreads, F f)
{
    std::vector<std::thread> th;
    for (int t = 1; t < nthreads; ++t) th.emplace_back(f, t);
    f(0);
    for (auto& x : th) x.join();
}
}  // namespace

struct cpub_acq
{
    int N{0}, D{0}, P{0}, G{0}, DB{0};
    Plan plan;
    std::vector<std::complex<float>> wipe;  // D x N
    cv* code{nullptr};                      // G x N: FFT(code_p), lane = p % 8
    cv* X{nullptr};                         // DB x N: forward spectra, lane = d % 8
    std::vector<RowStat> stats;             // P x D
    int dmax{0}, dstep{0};
    ~cpub_acq()
    {
        free(code);
        free(X);
    }
};

extern "C" {

// acquisition batch of P PRNs (codes: P rows of N complex<float>, already placed in
// the FFT buffer as set_local_code does for consumed == fft_size), D bins from
// -dmax in steps of dstep.
cpub_acq* cpub_acq_create(int N, int D, int P, double fs, int dmax, int dstep, const float* codes)
{
    auto* a = new (std::nothrow) cpub_acq();
    if (!a) return nullptr;
    if (!a->plan.make(N))
        {
            delete a;
            return nullptr;
        }
    a->N = N;
    a->D = D;
    a->P = P;
    a->G = (P + 7) / 8;
    a->DB = (D + 7) / 8;
    a->dmax = dmax;
    a->dstep = dstep;
    // update_grid_doppler_wipeoffs (:298-305) with the generic sincos: phase
    // accumulated in fp32 from 0, then cos / sin of each phase
    a->wipe.resize(static_cast<size_t>(D) * N);
    for (int d = 0; d < D; ++d)
        {
            const float freq = (float)(-dmax + dstep * d);
            const float step = -(float)(2.0 * M_PI) * freq / (float)fs;
            float ph = 0.0f;
            for (int n = 0; n < N; ++n)
                {
                    a->wipe[static_cast<size_t>(d) * N + n] = std::complex<float>(std::cos(ph), std::sin(ph));
                    ph += step;
                }
        }
    a->code = static_cast<cv*>(aligned_alloc64(sizeof(cv) * static_cast<size_t>(a->G) * N));
    a->X = static_cast<cv*>(aligned_alloc64(sizeof(cv) * static_cast<size_t>(a->DB) * N));
    cv* tmp = static_cast<cv*>(aligned_alloc64(sizeof(cv) * N));
    if (!a->code || !a->X || !tmp)
        {
            free(tmp);
            delete a;
            return nullptr;
        }
    for (int g = 0; g < a->G; ++g)
        {
            cv* c = a->code + static_cast<size_t>(g) * N;
            for (int n = 0; n < N; ++n)
                for (int l = 0; l < 8; ++l)
                    {
                        const int p = g * 8 + l;
                        c[n].r[l] = p < P ? codes[(static_cast<size_t>(p) * N + n) * 2] : 0.0f;
                        c[n].i[l] = p < P ? codes[(static_cast<size_t>(p) * N + n) * 2 + 1] : 0.0f;
                    }
            cv* r = a->plan.run(c, tmp);
            if (r != c) std::memcpy(c, r, sizeof(cv) * N);
        }
    free(tmp);
    a->stats.resize(static_cast<size_t>(P) * D);
    return a;
}

void cpub_acq_destroy(cpub_acq* a) { delete a; }

// One block of N gr_complex samples over nthreads threads; out: P records of
// (doppler_index, code_phase, peak, input_power, test_statistic) as 5 floats.
int cpub_acq_run(cpub_acq* a, const float* iq, int nthreads, float* out)
{
    const int N = a->N, D = a->D, P = a->P;
    if (nthreads < 1) nthreads = 1;
    const auto* x = reinterpret_cast<const std::complex<float>*>(iq);
    // forward spectra, 8 Doppler rows per task
    std::atomic<int> next{0};
    parallel(nthreads, [&](int) {
        cv* buf = static_cast<cv*>(aligned_alloc64(sizeof(cv) * N));
        for (int b; (b = next.fetch_add(1)) < a->DB;)
            {
                cv* xb = a->X + static_cast<size_t>(b) * N;
                for (int n = 0; n < N; ++n)
                    for (int l = 0; l < 8; ++l)
                        {
                            const int d = std::min(b * 8 + l, D - 1);
                            const std::complex<float> v = x[n] * a->wipe[static_cast<size_t>(d) * N + n];
                            xb[n].r[l] = v.real();
                            xb[n].i[l] = v.imag();
                        }
                cv* r = a->plan.run(xb, buf);
                if (r != xb) std::memcpy(xb, r, sizeof(cv) * N);
            }
        free(buf);
    });
    // correlation rows: task = (d, PRN group of 8)
    next = 0;
    parallel(nthreads, [&](int) {
        cv* y = static_cast<cv*>(aligned_alloc64(sizeof(cv) * N));
        cv* buf = static_cast<cv*>(aligned_alloc64(sizeof(cv) * N));
        for (int t; (t = next.fetch_add(1)) < D * a->G;)
            {
                const int d = t / a->G, g = t % a->G;
                const cv* xb = a->X + static_cast<size_t>(d / 8) * N;
                const int l = d % 8;
                const cv* c = a->code + static_cast<size_t>(g) * N;
                // |IFFT(X . conj(C))| = |FFT(conj(X) . C)|
                for (int n = 0; n < N; ++n)
                    {
                        const float xr = xb[n].r[l], xi = xb[n].i[l];
                        y[n].r = xr * c[n].r + xi * c[n].i;
                        y[n].i = xr * c[n].i - xi * c[n].r;
                    }
                const cv* R = a->plan.run(y, buf);
                v8 best = bc(-1.0f), sum = bc(0.0f);
                v8i bidx = {0, 0, 0, 0, 0, 0, 0, 0};
                for (int n = 0; n < N; ++n)
                    {
                        const v8 m = R[n].r * R[n].r + R[n].i * R[n].i;
                        const v8i gt = m > best;  // strict '>': the first maximum (32f_index_max_32u)
                        best = gt ? m : best;
                        bidx = gt ? v8i{n, n, n, n, n, n, n, n} : bidx;
                        sum += m;
                    }
                for (int q = 0; q < 8; ++q)
                    {
                        const int p = g * 8 + q;
                        if (p < P) a->stats[static_cast<size_t>(p) * D + d] = RowStat{best[q], (uint32_t)bidx[q], sum[q]};
                    }
            }
        free(y);
        free(buf);
    });
    // max_to_input_power_statistic (:511-543) per PRN
    for (int p = 0; p < P; ++p)
        {
            const RowStat* s = &a->stats[static_cast<size_t>(p) * D];
            float gmax = 0.0f;
            int dsel = 0;
            uint32_t tsel = 0;
            for (int d = 0; d < D; ++d)
                if (s[d].max > gmax)
                    {
                        gmax = s[d].max;
                        dsel = d;
                        tsel = s[d].idx;
                    }
            const int opp = (dsel + D / 2) % D;
            const float ip = (float)((double)(s[opp].sum / (float)N) / 2.0 / 1.0);
            out[p * 5 + 0] = (float)dsel;
            out[p * 5 + 1] = (float)tsel;
            out[p * 5 + 2] = gmax;
            out[p * 5 + 3] = ip;
            out[p * 5 + 4] = gmax / ip;
        }
    return 0;
}

// Fused resampler + rotator dot product, AVX2 (real codes, K <= 5 taps): the
// Carrier_wipeoff_multicorrelator_resampler inputs (cpu_multicorrelator_real_codes.cc:
// 103-126); out: K complex.
void cpub_corr(float* out, const float* sig, const float* code, int L, const float* shifts, int K, float rem_carr,
    float carr_step, float rem_code, float code_step, int n)
{
    // phasors of samples n0 + {0,1,4,5,2,3,6,7}: the lane order of the
    // shuffle_ps de-interleave below
    static const int lane_off[8] = {0, 1, 4, 5, 2, 3, 6, 7};
    const std::complex<float> ph0(std::cos(rem_carr), -std::sin(rem_carr));
    const std::complex<float> inc(std::cos(carr_step), -std::sin(carr_step));
    std::complex<float> pw[8];
    pw[0] = std::complex<float>(1.0f, 0.0f);
    for (int k = 1; k < 8; ++k) pw[k] = pw[k - 1] * inc;
    const std::complex<float> inc8 = pw[7] * inc;
    v8 pr, pi;
    for (int l = 0; l < 8; ++l)
        {
            const std::complex<float> v = ph0 * pw[lane_off[l]];
            pr[l] = v.real();
            pi[l] = v.imag();
        }
    v8 accr[5], acci[5];
    v8 off[5];
    for (int k = 0; k < 5; ++k)
        {
            accr[k] = bc(0.0f);
            acci[k] = bc(0.0f);
            off[k] = bc(k < K ? shifts[k] - rem_code : 0.0f);
        }
    v8 nf;
    for (int l = 0; l < 8; ++l) nf[l] = (float)lane_off[l];
    const v8 stepv = bc(code_step);
    const __m256i Lv = _mm256_set1_epi32(L);
    const __m256i zero = _mm256_setzero_si256();
    int i = 0;
    for (; i + 8 <= n; i += 8)
        {
            const __m256 a = _mm256_loadu_ps(sig + 2 * i), b = _mm256_loadu_ps(sig + 2 * i + 8);
            const v8 xr = (v8)_mm256_shuffle_ps(a, b, 0x88), xi = (v8)_mm256_shuffle_ps(a, b, 0xDD);
            const v8 yr = xr * pr - xi * pi, yi = xr * pi + xi * pr;
            const v8 t = nf * stepv;
            for (int k = 0; k < K; ++k)
                {
                    __m256i idx = _mm256_cvttps_epi32(_mm256_floor_ps((__m256)(t + off[k])));
                    idx = _mm256_add_epi32(idx, _mm256_and_si256(_mm256_cmpgt_epi32(zero, idx), Lv));
                    idx = _mm256_sub_epi32(idx, _mm256_andnot_si256(_mm256_cmpgt_epi32(Lv, idx), Lv));
                    const v8 c = (v8)_mm256_i32gather_ps(code, idx, 4);
                    accr[k] += c * yr;
                    acci[k] += c * yi;
                }
            const v8 npr = pr * inc8.real() - pi * inc8.imag();
            pi = pr * inc8.imag() + pi * inc8.real();
            pr = npr;
            nf += bc(8.0f);
            if ((i & 255) == 248)
                {
                    // renormalise every 256 samples (the generic rotator's cadence)
                    const v8 mag = pr * pr + pi * pi;
                    const v8 inv = (v8)_mm256_div_ps(_mm256_set1_ps(1.0f), _mm256_sqrt_ps((__m256)mag));
                    pr *= inv;
                    pi *= inv;
                }
        }
    float res[10] = {0};
    for (int k = 0; k < K; ++k)
        for (int l = 0; l < 8; ++l)
            {
                res[2 * k] += accr[k][l];
                res[2 * k + 1] += acci[k][l];
            }
    // scalar tail
    std::complex<float> ph = ph0;
    for (int s = 0; s < i; s += 8) ph *= inc8;
    for (; i < n; ++i)
        {
            const std::complex<float> y = std::complex<float>(sig[2 * i], sig[2 * i + 1]) * ph;
            for (int k = 0; k < K; ++k)
                {
                    int idx = (int)std::floor(code_step * (float)i + (shifts[k] - rem_code));
                    idx = ((idx % L) + L) % L;
                    res[2 * k] += code[idx] * y.real();
                    res[2 * k + 1] += code[idx] * y.imag();
                }
            ph *= inc;
        }
    for (int k = 0; k < 2 * K; ++k) out[k] = res[k];
}

// One dll_pll_veml_tracking call of an oracle channel with the AVX2 correlator
// (non-high-dynamics channels; others run the oracle's own correlator).
int cpub_trk_call(orc_trk* t, const float* in, uint64_t nitems_read, gsdr_trk_epoch* r)
{
    float p[6], shifts[5];
    int n = 0, L = 0;
    const float* code = nullptr;
    const int K = orc_trk_corr_params(t, p, &n, &code, &L, shifts);
    if (p[2] != 0.0f || p[5] != 0.0f) return orc_trk_call(t, in, nitems_read, r);
    float taps[12] = {0};
    cpub_corr(taps, in, code, L, shifts, K, p[0], p[1], p[3], p[4], n);
    return orc_trk_call_taps(t, taps, nitems_read, r);
}

// Tracking calls of nch channels over the same input in parallel: channel c reads
// iq from item data_off[c] on, its absolute input position being nitems_read[c];
// out: nch records.
void cpub_trk_calls(orc_trk** chans, int nch, const float* iq, const uint64_t* data_off, const uint64_t* nitems_read,
    int nthreads, gsdr_trk_epoch* out)
{
    std::atomic<int> next{0};
    parallel(std::max(1, std::min(nthreads, nch)), [&](int) {
        for (int c; (c = next.fetch_add(1)) < nch;)
            cpub_trk_call(chans[c], iq + 2 * data_off[c], nitems_read[c], &out[c]);
    });
}
}
