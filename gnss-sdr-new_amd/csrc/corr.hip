// Tracking multicorrelator engine for MI355X (gfx950).
//
// One fused launch replaces, for every job (channel-epoch) of a batch, the pair
//   volk_gnsssdr_32f_xn_resampler_32f_xn            (K code replicas written to memory)
//   volk_gnsssdr_32fc_32f_rotator_dot_prod_32fc_xn  (carrier rotator + K dot products)
// behind Cpu_Multicorrelator_Real_Codes::Carrier_wipeoff_multicorrelator_resampler
// (src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.cc:103-144), and the
// complex-replica pair behind Cpu_Multicorrelator (cpu_multicorrelator.cc:73-100).
//
// Per workgroup (one job): the channel's code replica is staged in LDS; each lane
// streams IQ samples (coalesced), regenerates the carrier phasor from an fp64
// phase (the reference's phasor recursion with its float-rounded phase_inc, but
// without its accumulated rounding), computes every tap's code index with the
// reference's exact float association (no FMA contraction), and
// accumulates K complex sums in VGPRs; wave64 shuffles + an LDS pass reduce them.
// The K x N resampled-code matrix of the reference never exists.
#include <hip/hip_runtime.h>

#include <cmath>
#include <complex>
#include <mutex>
#include <new>
#include <vector>

#include "gsdr_internal.h"

namespace
{

constexpr int kMaxTaps = 8;
constexpr int kCorrThreads = 256;
constexpr int kSamplesPerThread = 16;
constexpr int kChunk = kCorrThreads * kSamplesPerThread;  // samples per workgroup
constexpr int kMaxCodeSamples = 16384;                    // replica length limit (floats; complex codes 2x)
constexpr int kSpanCap = 4096;                            // LDS-staged replica span per chunk (entries)

struct ChanDev
{
    const float* code;  // L floats (real) or 2L floats (complex)
    int32_t L;
    int32_t ntaps;
    int32_t high_dyn;
    int32_t cplx;
    float shifts[kMaxTaps];
};

// Host-derived rotator model of one job (the reference builds phase_offset and
// phase_inc on the host too, cpu_multicorrelator_real_codes.cc:114-123).
struct JobAux
{
    double psi0;   // arg(cos(rem), -sin(rem)) in float
    double theta;  // arg(exp(-j*step)) in float
    double theta_rate;
    int32_t valid;
    int32_t pad;
};

template <int IT>
__device__ __forceinline__ float2 load_item(const void* __restrict__ p, int64_t i)
{
    if constexpr (IT == GSDR_ITEM_GR_COMPLEX)
        {
            return reinterpret_cast<const float2*>(p)[i];
        }
    else if constexpr (IT == GSDR_ITEM_CSHORT)
        {
            short2 s = reinterpret_cast<const short2*>(p)[i];
            return make_float2((float)s.x, (float)s.y);
        }
    else
        {
            // Ibyte_To_Complex: interleaved_char_to_complex, scale 1 (exact)
            char2 s = reinterpret_cast<const char2*>(p)[i];
            return make_float2((float)s.x, (float)s.y);
        }
}

__device__ __forceinline__ int wrap_mod(int idx, int L)
{
    int r = idx % L;
    return r < 0 ? r + L : r;
}

// KERN/32f_xn_resampler_32f_xn.h:73 (generic) / :384-390 (a_avx).
__device__ __forceinline__ int code_index(float step, float shift, float rem, int n, int L, int assoc)
{
    const float a = gsdr::mul_rn(step, (float)n);
    float t;
    if (assoc == GSDR_ASSOC_GENERIC)
        t = gsdr::sub_rn(gsdr::add_rn(a, shift), rem);
    else
        t = gsdr::add_rn(a, gsdr::sub_rn(shift, rem));
    return wrap_mod((int)floorf(t), L);
}

// KERN/32f_xn_high_dynamics_resampler_32f_xn.h:75-79 (tap 0).
__device__ __forceinline__ int code_index_hd(float step, float rate, float shift0, float rem, uint32_t m, int L)
{
    const float a = gsdr::mul_rn(step, (float)m);
    const float b = gsdr::mul_rn(rate, (float)(m * m));
    const float t = gsdr::sub_rn(gsdr::add_rn(gsdr::add_rn(a, b), shift0), rem);
    return wrap_mod((int)floorf(t), L);
}

__device__ __forceinline__ void rotator_model_device(const gsdr_corr_job& j, double& psi0, double& th, double& thr)
{
    float s, c;
    sincosf(j.rem_carr_phase_rad, &s, &c);
    psi0 = atan2(-(double)s, (double)c);
    sincosf(-j.carr_phase_step_rad, &s, &c);
    th = atan2((double)s, (double)c);
    sincosf(-j.carr_phase_rate_step_rad, &s, &c);
    thr = atan2((double)s, (double)c);
}

// Unwrapped code index floor(...) with the reference's float association.
__device__ __forceinline__ int raw_index(float step, float shift, float rem, int n, int assoc)
{
    const float a = gsdr::mul_rn(step, (float)n);
    const float t = (assoc == GSDR_ASSOC_GENERIC) ? gsdr::sub_rn(gsdr::add_rn(a, shift), rem) : gsdr::add_rn(a, gsdr::sub_rn(shift, rem));
    return (int)floorf(t);
}

// Span staging modes of one chunk's replica.
enum SpanMode
{
    kSpanLds = 1,     // code[(lo + i) mod L] staged in LDS, lookup s_code[raw - lo]
    kSpanGlobal = 2,  // lookup the replica in global memory (L1/L2-resident) with the modulo
};

// Streaming body of one chunk: lane-interleaved samples (coalesced loads), the carrier
// phasor anchored once per lane in fp64 and advanced by exp(j*theta*kCorrThreads),
// K taps accumulated in VGPRs.
template <int IT, bool CPLX, bool HD>
__device__ __forceinline__ void chunk_accumulate(const gsdr_corr_job& job, const ChanDev& ch, const float* s_code,
    int mode, int lo, const int* s_hdshift, double psi0, double th, double thr, float2 wstep, int n0, int n1,
    const float2 (&xs)[kSamplesPerThread], int assoc, float2 (*s_red)[kMaxTaps])
{
    float2 acc[kMaxTaps];
#pragma unroll
    for (int k = 0; k < kMaxTaps; ++k) acc[k] = make_float2(0.f, 0.f);
    const int L = ch.L;
    const int K = ch.ntaps;
    const int N = job.n_samples;
    const float rem = job.rem_code_phase_chips, step = job.code_phase_step_chips, rate = job.code_phase_rate_step_chips;
    constexpr double kTwoPi = 6.283185307179586476925286766559;
    constexpr double kInvTwoPi = 0.15915494309189533576888376337251;
    const float* code_g = ch.code;
    float2 ph = make_float2(1.f, 0.f);
    if (!HD)
        {
            const double phi = psi0 + (double)(n0 + (int)threadIdx.x) * th;
            const float a = (float)fma(-rint(phi * kInvTwoPi), kTwoPi, phi);
            float sn, cs;
            sincosf(a, &sn, &cs);
            ph = make_float2(cs, sn);
        }
#pragma unroll
    for (int it = 0; it < kSamplesPerThread; ++it)
        {
            const int n = n0 + (int)threadIdx.x + it * kCorrThreads;
            if (n < n1)
                {
                    const float2 x = xs[it];
                    float2 r = ph;
                    if (HD)
                        {
                            double phi = psi0 + (double)n * th;
                            if (n > 0)
                                {
                                    const double m1 = (double)(n - 1);
                                    phi += m1 * m1 * thr;
                                }
                            const float a = (float)fma(-rint(phi * kInvTwoPi), kTwoPi, phi);
                            float sn, cs;
                            sincosf(a, &sn, &cs);
                            r = make_float2(cs, sn);
                        }
                    const float2 t = make_float2(x.x * r.x - x.y * r.y, x.x * r.y + x.y * r.x);
#pragma unroll
                    for (int k = 0; k < kMaxTaps; ++k)
                        {
                            if (k < K)
                                {
                                    float cr, ci = 0.0f;
                                    if (HD)
                                        {
                                            const uint32_t m = (uint32_t)((n + s_hdshift[k]) % N);
                                            const int idx = code_index_hd(step, rate, ch.shifts[0], rem, m, L);
                                            cr = CPLX ? code_g[2 * idx] : code_g[idx];
                                            if (CPLX) ci = code_g[2 * idx + 1];
                                        }
                                    else
                                        {
                                            const int raw = raw_index(step, ch.shifts[k], rem, n, assoc);
                                            if (mode == kSpanLds)
                                                {
                                                    const int i = raw - lo;
                                                    cr = CPLX ? s_code[2 * i] : s_code[i];
                                                    if (CPLX) ci = s_code[2 * i + 1];
                                                }
                                            else
                                                {
                                                    const int idx = wrap_mod(raw, L);
                                                    cr = CPLX ? code_g[2 * idx] : code_g[idx];
                                                    if (CPLX) ci = code_g[2 * idx + 1];
                                                }
                                        }
                                    if (CPLX)
                                        {
                                            acc[k].x += t.x * cr - t.y * ci;
                                            acc[k].y += t.x * ci + t.y * cr;
                                        }
                                    else
                                        {
                                            acc[k].x += t.x * cr;
                                            acc[k].y += t.y * cr;
                                        }
                                }
                        }
                }
            if (!HD) ph = make_float2(ph.x * wstep.x - ph.y * wstep.y, ph.x * wstep.y + ph.y * wstep.x);
        }
    // wave64 reduction into s_red[wave]: DPP sums, the total in lane 63
#pragma unroll
    for (int k = 0; k < kMaxTaps; ++k)
        {
            acc[k].x = gsdr::wave_sum_lane63(acc[k].x);
            acc[k].y = gsdr::wave_sum_lane63(acc[k].y);
        }
    if ((threadIdx.x & 63) == 63)
        {
#pragma unroll
            for (int k = 0; k < kMaxTaps; ++k) s_red[threadIdx.x >> 6][k] = acc[k];
        }
}

// grid = (chunks, jobs).  Workgroup (c, j) correlates samples [c*kChunk, (c+1)*kChunk)
// of job j; the last workgroup of a job to finish sums the chunk partials in chunk
// order (deterministic) and writes the K outputs.
template <int IT>
__global__ void __launch_bounds__(kCorrThreads) corr_kernel(const gsdr_corr_job* __restrict__ jobs,
    const JobAux* __restrict__ aux, const ChanDev* __restrict__ chans, const void* __restrict__ iq, int64_t iq_items,
    float2* __restrict__ out, int max_taps, int assoc, float2* __restrict__ partials, unsigned int* __restrict__ counters,
    int max_chunks, int nchan)
{
    extern __shared__ float s_code[];
    __shared__ double s_model[3];
    __shared__ float2 s_wstep;
    __shared__ int s_hdshift[kMaxTaps];
    __shared__ int s_lo, s_span, s_mode, s_last;
    __shared__ float2 s_red[kCorrThreads / 64][kMaxTaps];

    const int jb = blockIdx.y, chunk = blockIdx.x;
    const gsdr_corr_job job = jobs[jb];
    // device-resident job tables are not validated by the host: a job whose channel
    // is out of range or whose length exceeds the handle's max_len (more chunks than
    // the grid holds) gets NaN outputs from chunk 0 and never touches the arrival
    // counter, so later launches' last-arriver detection stays intact
    if (job.channel < 0 || job.channel >= nchan || job.n_samples < 0 ||
        (job.n_samples + kChunk - 1) / kChunk > max_chunks)
        {
            if (chunk == 0 && (int)threadIdx.x < max_taps)
                out[(size_t)jb * max_taps + threadIdx.x] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
            return;
        }
    const ChanDev ch = chans[job.channel];
    const int K = ch.ntaps;
    const int N = job.n_samples;
    const int nchunks = N > 0 ? (N + kChunk - 1) / kChunk : 1;
    if (chunk >= nchunks) return;
    const int n0 = chunk * kChunk;
    const int n1 = min(N, n0 + kChunk);
    const bool hd = ch.high_dyn != 0;

    // issue this lane's IQ loads first: they depend on the job only, so their
    // latency overlaps the replica-span staging below
    float2 xs[kSamplesPerThread];
#pragma unroll
    for (int it = 0; it < kSamplesPerThread; ++it)
        {
            const int n = n0 + (int)threadIdx.x + it * kCorrThreads;
            const int64_t item = job.sample_offset + n;
            xs[it] = (n < n1 && item >= 0 && item < iq_items) ? load_item<IT>(iq, item) : make_float2(0.f, 0.f);
        }

    if (threadIdx.x == 0)
        {
            double psi0, th, thr;
            if (aux && aux[jb].valid)
                {
                    psi0 = aux[jb].psi0;
                    th = aux[jb].theta;
                    thr = aux[jb].theta_rate;
                }
            else
                {
                    rotator_model_device(job, psi0, th, thr);
                }
            s_model[0] = psi0;
            s_model[1] = th;
            s_model[2] = thr;
            const double w = th * (double)kCorrThreads;
            float sn, cs;
            sincosf((float)fma(-rint(w * 0.15915494309189533576888376337251), 6.283185307179586476925286766559, w), &sn,
                &cs);
            s_wstep = make_float2(cs, sn);
            // high-dynamics taps 1..K-1 are sample-shifted copies of tap 0
            // (KERN/32f_xn_high_dynamics_resampler_32f_xn.h:84-91)
            unsigned int sh = 0;
            s_hdshift[0] = 0;
#pragma unroll
            for (int k = 1; k < kMaxTaps; ++k)
                {
                    if (k < K) sh += (int)roundf((ch.shifts[k] - ch.shifts[k - 1]) / job.code_phase_step_chips);
                    s_hdshift[k] = (int)sh;
                }
            // replica span of this chunk: the index is monotone in n for step > 0
            int mode = kSpanGlobal, lo = 0, span = 0;
            const float step = job.code_phase_step_chips, rem = job.rem_code_phase_chips;
            if (!hd && step > 0.0f && n1 > n0)
                {
                    int mn = INT_MAX, mx = INT_MIN;
#pragma unroll
                    for (int k = 0; k < kMaxTaps; ++k)
                        {
                            if (k < K)
                                {
                                    mn = min(mn, raw_index(step, ch.shifts[k], rem, n0, assoc));
                                    mx = max(mx, raw_index(step, ch.shifts[k], rem, n1 - 1, assoc));
                                }
                        }
                    if (mx >= mn && mx - mn + 1 <= kSpanCap)
                        {
                            mode = kSpanLds;
                            lo = mn;
                            span = mx - mn + 1;
                        }
                }
            s_mode = mode;
            s_lo = lo;
            s_span = span;
        }
    __syncthreads();
    const int mode = s_mode, lo = s_lo, span = s_span, L = ch.L;
    if (mode == kSpanLds)
        {
            if (ch.cplx)
                {
                    for (int i = threadIdx.x; i < span; i += kCorrThreads)
                        {
                            const int idx = wrap_mod(lo + i, L);
                            s_code[2 * i] = ch.code[2 * idx];
                            s_code[2 * i + 1] = ch.code[2 * idx + 1];
                        }
                }
            else
                {
                    for (int i = threadIdx.x; i < span; i += kCorrThreads) s_code[i] = ch.code[wrap_mod(lo + i, L)];
                }
        }
    __syncthreads();

    const double psi0 = s_model[0], th = s_model[1], thr = s_model[2];
    const float2 ws = s_wstep;
    if (hd)
        {
            if (ch.cplx)
                chunk_accumulate<IT, true, true>(job, ch, s_code, mode, lo, s_hdshift, psi0, th, thr, ws, n0, n1, xs,
                    assoc, s_red);
            else
                chunk_accumulate<IT, false, true>(job, ch, s_code, mode, lo, s_hdshift, psi0, th, thr, ws, n0, n1, xs,
                    assoc, s_red);
        }
    else
        {
            if (ch.cplx)
                chunk_accumulate<IT, true, false>(job, ch, s_code, mode, lo, s_hdshift, psi0, th, thr, ws, n0, n1, xs,
                    assoc, s_red);
            else
                chunk_accumulate<IT, false, false>(job, ch, s_code, mode, lo, s_hdshift, psi0, th, thr, ws, n0, n1, xs,
                    assoc, s_red);
        }

    const int wave = threadIdx.x >> 6;
    __syncthreads();
    if (nchunks == 1)
        {
            if (threadIdx.x < K)
                {
                    float2 r = make_float2(0.f, 0.f);
#pragma unroll
                    for (int w = 0; w < kCorrThreads / 64; ++w)
                        {
                            r.x += s_red[w][threadIdx.x].x;
                            r.y += s_red[w][threadIdx.x].y;
                        }
                    out[(size_t)jb * max_taps + threadIdx.x] = r;
                }
            return;
        }
    // cross-chunk hand-off without cache-maintenance fences (MI355X_MICROARCH.md,
    // "Valid forms", table row 1): wave 0 writes its partials with agent-scope
    // (sc1, write-through) stores, drains them, then one lane arrives on the job's
    // counter with an agent-scope atomic; the last arriver reads every partial with
    // agent-scope (sc1) loads after its atomic has returned.
    if (wave == 0)
        {
            if (threadIdx.x < K)
                {
                    float2 r = make_float2(0.f, 0.f);
#pragma unroll
                    for (int w = 0; w < kCorrThreads / 64; ++w)
                        {
                            r.x += s_red[w][threadIdx.x].x;
                            r.y += s_red[w][threadIdx.x].y;
                        }
                    unsigned long long bits;
                    __builtin_memcpy(&bits, &r, sizeof(bits));
                    __hip_atomic_store(reinterpret_cast<unsigned long long*>(
                                           &partials[((size_t)jb * max_chunks + chunk) * kMaxTaps + threadIdx.x]),
                        bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            if (threadIdx.x == 0)
                {
                    const unsigned int prev =
                        __hip_atomic_fetch_add(&counters[jb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    s_last = (prev == (unsigned int)(nchunks - 1)) ? 1 : 0;
                }
        }
    __syncthreads();
    if (!s_last) return;
    if (threadIdx.x < K)
        {
            float2 r = make_float2(0.f, 0.f);
            for (int c = 0; c < nchunks; ++c)
                {
                    const unsigned long long bits = __hip_atomic_load(reinterpret_cast<unsigned long long*>(
                                                                          &partials[((size_t)jb * max_chunks + c) * kMaxTaps + threadIdx.x]),
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    float2 v;
                    __builtin_memcpy(&v, &bits, sizeof(v));
                    r.x += v.x;
                    r.y += v.y;
                }
            out[(size_t)jb * max_taps + threadIdx.x] = r;
        }
    if (threadIdx.x == 0) counters[jb] = 0u;  // re-armed for the next launch on this stream
}

__global__ void corr_index_kernel(const ChanDev* __restrict__ chans, int channel, float rem, float step, int n_total,
    int assoc, int32_t* __restrict__ out)
{
    const ChanDev ch = chans[channel];
    const int n = blockIdx.x * blockDim.x + threadIdx.x;
    if (n >= n_total) return;
    for (int k = 0; k < ch.ntaps; ++k) out[(size_t)k * n_total + n] = code_index(step, ch.shifts[k], rem, n, ch.L, assoc);
}

}  // namespace

struct gsdr_corr
{
    int device{0};
    int max_channels{0}, max_len{0}, max_taps{0};
    int assoc{GSDR_ASSOC_AVX};
    hipStream_t stream{nullptr};
    std::vector<ChanDev> chans;       // host mirror of the descriptors
    std::vector<float*> code_bufs;    // per-channel device replica buffers
    std::vector<int> code_caps;
    ChanDev* d_chans{nullptr};
    gsdr_corr_job* d_jobs{nullptr};
    JobAux* d_aux{nullptr};
    float2* d_partials{nullptr};      // jobs_cap x max_chunks x kMaxTaps chunk partial sums
    unsigned int* d_counters{nullptr};  // per-job arrival counters (self re-arming)
    int max_chunks{1};
    int jobs_cap{0};
    void* d_iq{nullptr};
    float2* d_out{nullptr};
    std::vector<JobAux> h_aux;
    int max_code_floats{0};  // largest staged replica over configured channels (sizes the LDS)
    bool profiling{false};
    std::vector<std::pair<hipEvent_t, hipEvent_t>> prof_recs;
    std::vector<hipEvent_t> prof_pool;
    std::mutex mu;
};

namespace
{

size_t item_bytes(int it) { return it == GSDR_ITEM_CSHORT ? 4 : (it == GSDR_ITEM_IBYTE ? 2 : 8); }

// The reference's host-side phasors, bit for bit (std::cos/std::sin/std::exp on
// float, cpu_multicorrelator_real_codes.cc:114-123), reduced to their angles.
JobAux host_model(const gsdr_corr_job& j)
{
    JobAux a{};
    const std::complex<float> off(std::cos(j.rem_carr_phase_rad), -std::sin(j.rem_carr_phase_rad));
    const std::complex<float> inc = std::exp(std::complex<float>(0.0f, -j.carr_phase_step_rad));
    const std::complex<float> rate = std::exp(std::complex<float>(0.0f, -j.carr_phase_rate_step_rad));
    a.psi0 = std::atan2((double)off.imag(), (double)off.real());
    a.theta = std::atan2((double)inc.imag(), (double)inc.real());
    a.theta_rate = std::atan2((double)rate.imag(), (double)rate.real());
    a.valid = 1;
    return a;
}

int ensure_jobs(gsdr_corr* c, int njobs)
{
    if (njobs <= c->jobs_cap) return GSDR_OK;
    int cap = c->jobs_cap ? c->jobs_cap : 64;
    while (cap < njobs) cap *= 2;
    void* bufs[] = {c->d_jobs, c->d_aux, c->d_partials, c->d_counters};
    for (void* p : bufs)
        if (p) GSDR_HIP(hipFree(p));
    c->d_jobs = nullptr;
    c->d_aux = nullptr;
    c->d_partials = nullptr;
    c->d_counters = nullptr;
    c->jobs_cap = 0;
    GSDR_HIP(hipMalloc(&c->d_jobs, cap * sizeof(gsdr_corr_job)));
    GSDR_HIP(hipMalloc(&c->d_aux, cap * sizeof(JobAux)));
    GSDR_HIP(hipMalloc(&c->d_partials, (size_t)cap * c->max_chunks * kMaxTaps * sizeof(float2)));
    GSDR_HIP(hipMalloc(&c->d_counters, cap * sizeof(unsigned int)));
    GSDR_HIP(hipMemset(c->d_counters, 0, cap * sizeof(unsigned int)));
    c->jobs_cap = cap;
    return GSDR_OK;
}

int launch(gsdr_corr* c, const gsdr_corr_job* d_jobs, const JobAux* d_aux, int njobs, const void* iq, int item_type,
    int64_t iq_items, float* out, hipStream_t s)
{
    if (njobs == 0) return GSDR_OK;
    int rc = ensure_jobs(c, njobs);  // partial/counter workspace sized for this batch
    if (rc != GSDR_OK) return rc;
    const size_t lds = (size_t)2 * kSpanCap * sizeof(float);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->profiling)
        {
            for (hipEvent_t* e : {&e0, &e1})
                {
                    if (!c->prof_pool.empty())
                        {
                            *e = c->prof_pool.back();
                            c->prof_pool.pop_back();
                        }
                    else
                        GSDR_HIP(hipEventCreate(e));
                }
            GSDR_HIP(hipEventRecord(e0, s));
        }
    const dim3 grid(c->max_chunks, njobs);
    if (item_type == GSDR_ITEM_GR_COMPLEX)
        hipLaunchKernelGGL((corr_kernel<GSDR_ITEM_GR_COMPLEX>), grid, dim3(kCorrThreads), lds, s, d_jobs, d_aux,
            c->d_chans, iq, iq_items, (float2*)out, c->max_taps, c->assoc, c->d_partials, c->d_counters, c->max_chunks, c->max_channels);
    else if (item_type == GSDR_ITEM_CSHORT)
        hipLaunchKernelGGL((corr_kernel<GSDR_ITEM_CSHORT>), grid, dim3(kCorrThreads), lds, s, d_jobs, d_aux,
            c->d_chans, iq, iq_items, (float2*)out, c->max_taps, c->assoc, c->d_partials, c->d_counters, c->max_chunks, c->max_channels);
    else
        hipLaunchKernelGGL((corr_kernel<GSDR_ITEM_IBYTE>), grid, dim3(kCorrThreads), lds, s, d_jobs, d_aux,
            c->d_chans, iq, iq_items, (float2*)out, c->max_taps, c->assoc, c->d_partials, c->d_counters, c->max_chunks, c->max_channels);
    GSDR_HIP(hipGetLastError());
    if (c->profiling)
        {
            GSDR_HIP(hipEventRecord(e1, s));
            c->prof_recs.push_back({e0, e1});
        }
    return GSDR_OK;
}

int set_code_common(gsdr_corr* c, int ch, int L, const float* code, const float* shifts, int ntaps, int cplx)
{
    GSDR_REQUIRE(c && code && shifts, GSDR_E_ARG, "set_local_code_and_taps: null argument");
    GSDR_REQUIRE(ch >= 0 && ch < c->max_channels, GSDR_E_ARG, "set_local_code_and_taps: channel %d outside [0,%d)", ch,
        c->max_channels);
    GSDR_REQUIRE(ntaps >= 1 && ntaps <= c->max_taps, GSDR_E_ARG, "set_local_code_and_taps: %d taps outside [1,%d]", ntaps,
        c->max_taps);
    const int floats = cplx ? 2 * L : L;
    GSDR_REQUIRE(L >= 1 && floats <= 2 * kMaxCodeSamples, GSDR_E_UNSUPPORTED,
        "set_local_code_and_taps: code length %d outside the LDS-staged capacity", L);
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    if (c->code_caps[ch] < floats)
        {
            if (c->code_bufs[ch]) GSDR_HIP(hipFree(c->code_bufs[ch]));
            c->code_bufs[ch] = nullptr;
            c->code_caps[ch] = 0;
            GSDR_HIP(hipMalloc(&c->code_bufs[ch], floats * sizeof(float)));
            c->code_caps[ch] = floats;
        }
    GSDR_HIP(hipMemcpyAsync(c->code_bufs[ch], code, floats * sizeof(float), hipMemcpyHostToDevice, c->stream));
    ChanDev& d = c->chans[ch];
    d.code = c->code_bufs[ch];
    d.L = L;
    d.ntaps = ntaps;
    d.cplx = cplx;
    for (int k = 0; k < kMaxTaps; ++k) d.shifts[k] = k < ntaps ? shifts[k] : 0.0f;
    if (floats > c->max_code_floats) c->max_code_floats = floats;
    GSDR_HIP(hipMemcpyAsync(c->d_chans + ch, &d, sizeof(ChanDev), hipMemcpyHostToDevice, c->stream));
    GSDR_HIP(hipStreamSynchronize(c->stream));
    return GSDR_OK;
}

}  // namespace

extern "C" {

int gsdr_corr_create(int device, int max_channels, int max_len, int max_taps, gsdr_corr** out)
{
    GSDR_REQUIRE(out, GSDR_E_ARG, "gsdr_corr_create: null argument");
    *out = nullptr;
    GSDR_REQUIRE(max_channels > 0 && max_len > 0, GSDR_E_ARG, "gsdr_corr_create: capacities must be > 0");
    GSDR_REQUIRE(max_taps >= 1 && max_taps <= kMaxTaps, GSDR_E_UNSUPPORTED, "gsdr_corr_create: max_taps %d outside [1,%d]",
        max_taps, kMaxTaps);
    int ndev = 0;
    GSDR_HIP(hipGetDeviceCount(&ndev));
    GSDR_REQUIRE(device >= 0 && device < ndev, GSDR_E_ARG, "gsdr_corr_create: device %d of %d", device, ndev);
    gsdr::DeviceGuard g(device);
    gsdr_corr* c = new (std::nothrow) gsdr_corr();
    GSDR_REQUIRE(c, GSDR_E_ALLOC, "gsdr_corr_create: out of host memory");
    c->device = device;
    c->max_channels = max_channels;
    c->max_len = max_len;
    c->max_taps = max_taps;
    c->max_chunks = (max_len + kChunk - 1) / kChunk;
    c->chans.assign(max_channels, ChanDev{});
    for (auto& d : c->chans) d.ntaps = 0;
    c->code_bufs.assign(max_channels, nullptr);
    c->code_caps.assign(max_channels, 0);
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&c->d_chans, max_channels * sizeof(ChanDev));
    if (e == hipSuccess) e = hipMemset(c->d_chans, 0, max_channels * sizeof(ChanDev));
    if (e == hipSuccess) e = hipMalloc(&c->d_iq, (size_t)max_len * 8);
    if (e == hipSuccess) e = hipMalloc(&c->d_out, (size_t)max_taps * sizeof(float2));
    if (e != hipSuccess)
        {
            gsdr::set_error("gsdr_corr_create: %s", hipGetErrorString(e));
            gsdr_corr_destroy(c);
            return GSDR_E_ALLOC;
        }
    const size_t lds = (size_t)2 * kSpanCap * sizeof(float);
    GSDR_HIP(hipFuncSetAttribute((const void*)corr_kernel<GSDR_ITEM_GR_COMPLEX>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    GSDR_HIP(hipFuncSetAttribute((const void*)corr_kernel<GSDR_ITEM_CSHORT>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    GSDR_HIP(hipFuncSetAttribute((const void*)corr_kernel<GSDR_ITEM_IBYTE>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    if (ensure_jobs(c, 64) != GSDR_OK)
        {
            gsdr_corr_destroy(c);
            return GSDR_E_ALLOC;
        }
    *out = c;
    return GSDR_OK;
}

void gsdr_corr_destroy(gsdr_corr* c)
{
    if (!c) return;
    gsdr::DeviceGuard g(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    for (auto& r : c->prof_recs)
        {
            (void)hipEventDestroy(r.first);
            (void)hipEventDestroy(r.second);
        }
    for (hipEvent_t e : c->prof_pool) (void)hipEventDestroy(e);
    for (float* p : c->code_bufs)
        if (p) (void)hipFree(p);
    void* bufs[] = {c->d_chans, c->d_jobs, c->d_aux, c->d_partials, c->d_counters, c->d_iq, c->d_out};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int gsdr_corr_set_local_code_and_taps(gsdr_corr* c, int ch, int L, const float* code, const float* shifts, int ntaps)
{
    return set_code_common(c, ch, L, code, shifts, ntaps, 0);
}

int gsdr_corr_set_local_code_and_taps_complex(gsdr_corr* c, int ch, int L, const float* code, const float* shifts,
    int ntaps)
{
    return set_code_common(c, ch, L, code, shifts, ntaps, 1);
}

int gsdr_corr_set_high_dynamics_resampler(gsdr_corr* c, int ch, int enable)
{
    GSDR_REQUIRE(c, GSDR_E_ARG, "set_high_dynamics_resampler: null handle");
    GSDR_REQUIRE(ch >= 0 && ch < c->max_channels, GSDR_E_ARG, "set_high_dynamics_resampler: channel %d", ch);
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    c->chans[ch].high_dyn = enable ? 1 : 0;
    GSDR_HIP(hipMemcpyAsync(c->d_chans + ch, &c->chans[ch], sizeof(ChanDev), hipMemcpyHostToDevice, c->stream));
    GSDR_HIP(hipStreamSynchronize(c->stream));
    return GSDR_OK;
}

int gsdr_corr_set_resampler_assoc(gsdr_corr* c, int assoc)
{
    GSDR_REQUIRE(c, GSDR_E_ARG, "set_resampler_assoc: null handle");
    GSDR_REQUIRE(assoc == GSDR_ASSOC_GENERIC || assoc == GSDR_ASSOC_AVX, GSDR_E_ARG, "set_resampler_assoc: %d", assoc);
    c->assoc = assoc;
    return GSDR_OK;
}

int gsdr_corr_run_batch(gsdr_corr* c, const gsdr_corr_job* jobs, int njobs, const void* iq_dev, int item_type,
    int64_t iq_items, float* out_dev, void* stream)
{
    GSDR_REQUIRE(c && (jobs || njobs == 0) && iq_dev && out_dev, GSDR_E_ARG, "gsdr_corr_run_batch: null argument");
    GSDR_REQUIRE(item_type >= GSDR_ITEM_GR_COMPLEX && item_type <= GSDR_ITEM_IBYTE, GSDR_E_ARG,
        "gsdr_corr_run_batch: item type %d", item_type);
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    c->h_aux.resize(njobs);
    for (int j = 0; j < njobs; ++j)
        {
            const gsdr_corr_job& jb = jobs[j];
            GSDR_REQUIRE(jb.channel >= 0 && jb.channel < c->max_channels && c->chans[jb.channel].ntaps > 0, GSDR_E_STATE,
                "gsdr_corr_run_batch: job %d uses channel %d without a local code", j, jb.channel);
            GSDR_REQUIRE(jb.n_samples >= 0 && jb.n_samples <= c->max_len, GSDR_E_ARG,
                "gsdr_corr_run_batch: job %d length %d outside [0,%d]", j, jb.n_samples, c->max_len);
            c->h_aux[j] = host_model(jb);
        }
    int rc = ensure_jobs(c, njobs);
    if (rc != GSDR_OK) return rc;
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    GSDR_HIP(hipMemcpyAsync(c->d_jobs, jobs, njobs * sizeof(gsdr_corr_job), hipMemcpyHostToDevice, s));
    GSDR_HIP(hipMemcpyAsync(c->d_aux, c->h_aux.data(), njobs * sizeof(JobAux), hipMemcpyHostToDevice, s));
    return launch(c, c->d_jobs, c->d_aux, njobs, iq_dev, item_type, iq_items, out_dev, s);
}

int gsdr_corr_run_batch_device(gsdr_corr* c, const gsdr_corr_job* jobs_dev, int njobs, const void* iq_dev,
    int item_type, int64_t iq_items, float* out_dev, void* stream)
{
    GSDR_REQUIRE(c && (jobs_dev || njobs == 0) && iq_dev && out_dev, GSDR_E_ARG,
        "gsdr_corr_run_batch_device: null argument");
    gsdr::DeviceGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    return launch(c, jobs_dev, nullptr, njobs, iq_dev, item_type, iq_items, out_dev, s);
}

int gsdr_corr_run(gsdr_corr* c, int ch, const void* sig_in_host, int item_type, float rem_carr, float carr_step,
    float carr_rate, float rem_code, float code_step, float code_rate, int n, float* out_host)
{
    GSDR_REQUIRE(c && sig_in_host && out_host, GSDR_E_ARG, "gsdr_corr_run: null argument");
    GSDR_REQUIRE(n >= 0 && n <= c->max_len, GSDR_E_ARG, "gsdr_corr_run: length %d outside [0,%d]", n, c->max_len);
    GSDR_REQUIRE(ch >= 0 && ch < c->max_channels && c->chans[ch].ntaps > 0, GSDR_E_STATE,
        "gsdr_corr_run: channel %d has no local code", ch);
    GSDR_REQUIRE(item_type >= GSDR_ITEM_GR_COMPLEX && item_type <= GSDR_ITEM_IBYTE, GSDR_E_ARG,
        "gsdr_corr_run: item type %d", item_type);
    gsdr_corr_job jb{};
    jb.channel = ch;
    jb.n_samples = n;
    jb.sample_offset = 0;
    jb.rem_carr_phase_rad = rem_carr;
    jb.carr_phase_step_rad = carr_step;
    jb.carr_phase_rate_step_rad = carr_rate;
    jb.rem_code_phase_chips = rem_code;
    jb.code_phase_step_chips = code_step;
    jb.code_phase_rate_step_chips = code_rate;
    {
        std::lock_guard<std::mutex> lk(c->mu);
        gsdr::DeviceGuard g(c->device);
        GSDR_HIP(hipMemcpyAsync(c->d_iq, sig_in_host, (size_t)n * item_bytes(item_type), hipMemcpyHostToDevice,
            c->stream));
    }
    int rc = gsdr_corr_run_batch(c, &jb, 1, c->d_iq, item_type, n, (float*)c->d_out, c->stream);
    if (rc != GSDR_OK) return rc;
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    GSDR_HIP(hipMemcpyAsync(out_host, c->d_out, (size_t)c->chans[ch].ntaps * sizeof(float2), hipMemcpyDeviceToHost,
        c->stream));
    GSDR_HIP(hipStreamSynchronize(c->stream));
    return GSDR_OK;
}

int gsdr_corr_dump_indices(gsdr_corr* c, int ch, float rem, float step, int n, int32_t* idx_host)
{
    GSDR_REQUIRE(c && idx_host, GSDR_E_ARG, "gsdr_corr_dump_indices: null argument");
    GSDR_REQUIRE(ch >= 0 && ch < c->max_channels && c->chans[ch].ntaps > 0, GSDR_E_STATE,
        "gsdr_corr_dump_indices: channel %d has no local code", ch);
    GSDR_REQUIRE(n > 0, GSDR_E_ARG, "gsdr_corr_dump_indices: n must be > 0");
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    const int K = c->chans[ch].ntaps;
    int32_t* d_idx = nullptr;
    GSDR_HIP(hipMalloc(&d_idx, (size_t)K * n * sizeof(int32_t)));
    hipLaunchKernelGGL(corr_index_kernel, dim3((n + 255) / 256), dim3(256), 0, c->stream, c->d_chans, ch, rem, step, n,
        c->assoc, d_idx);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(idx_host, d_idx, (size_t)K * n * sizeof(int32_t), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_idx);
    GSDR_HIP(e);
    return GSDR_OK;
}

int gsdr_corr_run_epochs(gsdr_corr* c, const gsdr_corr_job* jobs_dev, int jobs_per_epoch, int n_epochs,
    const void* iq_dev, int item_type, int64_t iq_items, float* out_dev, void* stream)
{
    GSDR_REQUIRE(c && jobs_dev && iq_dev && out_dev, GSDR_E_ARG, "gsdr_corr_run_epochs: null argument");
    GSDR_REQUIRE(jobs_per_epoch >= 0 && n_epochs >= 0, GSDR_E_ARG, "gsdr_corr_run_epochs: negative count");
    GSDR_REQUIRE(item_type >= GSDR_ITEM_GR_COMPLEX && item_type <= GSDR_ITEM_IBYTE, GSDR_E_ARG,
        "gsdr_corr_run_epochs: item type %d", item_type);
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    hipStream_t s = stream ? (hipStream_t)stream : c->stream;
    for (int e = 0; e < n_epochs; ++e)
        {
            int rc = launch(c, jobs_dev + (size_t)e * jobs_per_epoch, nullptr, jobs_per_epoch, iq_dev, item_type, iq_items,
                out_dev + (size_t)2 * e * jobs_per_epoch * c->max_taps, s);
            if (rc != GSDR_OK) return rc;
        }
    return GSDR_OK;
}

int gsdr_corr_set_profiling(gsdr_corr* c, int enable)
{
    GSDR_REQUIRE(c, GSDR_E_ARG, "gsdr_corr_set_profiling: null handle");
    std::lock_guard<std::mutex> lk(c->mu);
    c->profiling = enable != 0;
    return GSDR_OK;
}

int gsdr_corr_read_profile(gsdr_corr* c, double* kernel_ms, uint32_t* launches)
{
    GSDR_REQUIRE(c && kernel_ms && launches, GSDR_E_ARG, "gsdr_corr_read_profile: null argument");
    std::lock_guard<std::mutex> lk(c->mu);
    gsdr::DeviceGuard g(c->device);
    *kernel_ms = 0.0;
    *launches = 0;
    for (auto& r : c->prof_recs)
        {
            GSDR_HIP(hipEventSynchronize(r.second));
            float ms = 0.0f;
            GSDR_HIP(hipEventElapsedTime(&ms, r.first, r.second));
            *kernel_ms += ms;
            *launches += 1;
            c->prof_pool.push_back(r.first);
            c->prof_pool.push_back(r.second);
        }
    c->prof_recs.clear();
    return GSDR_OK;
}

}  // extern "C"
