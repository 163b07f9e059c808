// Shared implementation of the PCPS acquisition engine (see acq.hip for the
// kernel map): kernels, the handle, launch templates.  Included by acq.hip (ABI)
// and by the variant translation units that instantiate the launch templates per
// FFT plan type, so the plan groups compile in parallel.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <type_traits>
#include <new>
#include <vector>

#include "fft_4step.h"
#include "fft_lds.h"
#include "fft_multi.h"
#include "fft_pk.h"
#include "fft_plan.h"
#include "gsdr_internal.h"

namespace
{

using gsdr::fft::Plan;


// Default correlate variant at N = 4000 (see GSDR_PK_VARIANTS).
constexpr int kDefaultCorrVariant4000 = 70;

// Default packed variant for an FFT size (0: none, the generic kernels).
inline int default_pk_variant(uint32_t N)
{
    switch (N)
        {
        case 4000: return kDefaultCorrVariant4000;
        case 16000: return 94;  // r04a: wave-local rows, +3 % over 93
        case 8000: return 61;
        case 2000: return 62;
        default: return 0;
        }
}

struct RowStat
{
    float max;
    uint32_t idx;
    float sum;
    uint32_t pad;
};

// Where the forward spectrum of (block-dwell bk, Doppler d) lives in d_X.  Doppler
// bins commensurate with the FFT bin spacing (doppler_step * N / fs = p / q in
// lowest terms, q <= D / 2) with the exact carrier (GSDR_WIPE_EXACT) make
// X_d[k] = X_{d mod q}[k + (d / q) p] an exact identity: the wipe-off of Doppler
// f + a q step is the one of f times exp(-j 2 pi a p n / N), a circular shift of
// the spectrum by a p bins.  The forward pass then computes only q spectra per
// block-dwell, each stored with its first E = ((D - 1) / q) p bins repeated after
// bin N - 1 (stride N + E), and every Doppler row is a window into one of them --
// no wrap arithmetic in the readers.  q = D, p = 0, stride = N is the plain layout
// (one spectrum per Doppler bin).
struct XMap
{
    uint32_t q;       // stored spectra per block-dwell
    uint32_t p;       // bin shift per class step
    uint32_t stride;  // complex elements per stored spectrum (N + E)
    __host__ __device__ __forceinline__ size_t off(uint32_t bk, uint32_t d) const
    {
        const uint32_t a = d / q, c = d - a * q;
        return ((size_t)bk * q + c) * stride + (size_t)a * p;
    }
};

struct AcqParams
{
    XMap xm;             // forward-spectrum layout (see XMap)
    uint32_t N;          // fft size
    uint32_t consumed;   // valid samples per block
    uint32_t lead_zeros; // zero samples placed before the code (sampled_ms != ms_per_code)
    uint32_t D;
    uint32_t P;
    int32_t doppler_max;
    int32_t doppler_center;
    int32_t doppler_step;
    float samples_per_code;
    uint32_t samples_per_chip;
    uint32_t dwells;      // max_dwells K (non-coherent dwells per acquisition attempt)
    float threshold;
    int32_t cfar;
    uint32_t eff;         // effective FFT size (N/2 with bit_transition_flag, else N)
    uint32_t out_off;     // first output index of the effective window (N - eff)
    // make_two_steps narrow grid (pcps_acquisition.cc:298-305, :533-540, :717-773)
    int32_t step_two;     // 1: Doppler from center2/step2, CFAR input power kept from the coarse step
    float center2;        // d_doppler_center_step_two
    float step2;          // Acq_Conf::doppler_step2
    float half2;          // static_cast<float>(floor(num_doppler_bins_step2 / 2.0))
    float ip2;            // d_input_power of the coarse step (not recomputed in step two, :530-540)
    uint32_t counter;     // d_num_noncoherent_integrations_counter of the statistic (CFAR divisor, :534)
};

// Acq_doppler_hz of Doppler row d: first step int32 arithmetic (:537); step two
// static_cast<int32_t>(center2 + (float(d) - half2) * step2) in float (:539).
__device__ __forceinline__ int32_t doppler_of(const AcqParams& ap, uint32_t d)
{
    if (ap.step_two) return (int32_t)gsdr::add_rn(ap.center2, gsdr::mul_rn(gsdr::sub_rn((float)d, ap.half2), ap.step2));
    return -ap.doppler_max + ap.doppler_center + ap.doppler_step * (int32_t)d;
}

template <int IT>
__device__ __forceinline__ float2 load_item(const void* __restrict__ p, size_t i)
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

__device__ __forceinline__ bool stat_better(float am, uint32_t ai, float bm, uint32_t bi)
{
    return am > bm || (am == bm && ai < bi);
}

// Block-wide (max, first argmax, sum) reduction; result valid in thread 0.
template <int NT>
__device__ __forceinline__ void block_reduce_stat(float& m, uint32_t& idx, float& sum, RowStat* scratch)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        {
            float om = __shfl_xor(m, off);
            uint32_t oi = __shfl_xor(idx, off);
            float os = __shfl_xor(sum, off);
            if (stat_better(om, oi, m, idx))
                {
                    m = om;
                    idx = oi;
                }
            sum += os;
        }
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (NW > 1)
        {
            if (lane == 0) scratch[wave] = RowStat{m, idx, sum, 0};
            __syncthreads();
            if (threadIdx.x == 0)
                {
                    for (int w = 1; w < NW; ++w)
                        {
                            RowStat s = scratch[w];
                            if (stat_better(s.max, s.idx, m, idx))
                                {
                                    m = s.max;
                                    idx = s.idx;
                                }
                            sum += s.sum;
                        }
                }
        }
}

// ---------------------------------------------------------------- K_wipe
// One workgroup per Doppler bin; the carrier model (GSDR_WIPE_*, gsdr.h):
//   EXACT   exp(-j 2 pi f n / fs) with the phase f n / fs reduced mod 1 in fp64 and
//           cos / sin in fp64, rounded once to fp32 (the default);
//   GENERIC the generic sincos protokernel (KERN/s32f_sincos_32fc.h:390-403): lane 0
//           replays the fp32 phase accumulation sequentially, the workgroup then
//           evaluates cosf / sinf in parallel;
//   AVX2    the a_avx2 protokernel (:448-627) the reference dispatches on AVX2 x86-64:
//           lanes 0..7 replay the eight fp32 accumulators (start phase + k inc, step
//           8 inc), the workgroup evaluates the Cephes polynomials in the kernel's fp32
//           operation order (no contraction), the N % 8 tail with cosf / sinf.
__device__ __forceinline__ float2 cephes_sincos_avx2(float x0)
{
    const float FOPI = 1.27323954473516f;
    const float DP1 = -0.78515625f, DP2 = -2.4187564849853515625e-4f, DP3 = -3.77489497744594108e-8f;
    const float C0 = 2.443315711809948E-005f, C1 = -1.388731625493765E-003f, C2 = 4.166664568298827E-002f;
    const float S0 = -1.9515295891E-4f, S1 = 8.3321608736E-3f, S2 = -1.6666654611E-1f;
    const uint32_t bits = __float_as_uint(x0);
    bool sign_sin = (bits >> 31) != 0;
    float x = __uint_as_float(bits & 0x7fffffffu);
    float y = __fmul_rn(x, FOPI);
    int32_t j = (int32_t)y;  // cvttps: truncation
    j = (j + 1) & ~1;
    y = (float)j;
    const bool swap = (j & 4) != 0;
    const bool poly = (j & 2) == 0;
    x = __fadd_rn(x, __fmul_rn(y, DP1));
    x = __fadd_rn(x, __fmul_rn(y, DP2));
    x = __fadd_rn(x, __fmul_rn(y, DP3));
    const bool sign_cos = ((~(j - 2)) & 4) != 0;
    sign_sin = sign_sin != swap;
    const float z = __fmul_rn(x, x);
    float yc = __fmul_rn(C0, z);
    yc = __fadd_rn(yc, C1);
    yc = __fmul_rn(yc, z);
    yc = __fadd_rn(yc, C2);
    yc = __fmul_rn(yc, z);
    yc = __fmul_rn(yc, z);
    yc = __fsub_rn(yc, __fmul_rn(z, 0.5f));
    yc = __fadd_rn(yc, 1.0f);
    float ys = __fmul_rn(S0, z);
    ys = __fadd_rn(ys, S1);
    ys = __fmul_rn(ys, z);
    ys = __fadd_rn(ys, S2);
    ys = __fmul_rn(ys, z);
    ys = __fmul_rn(ys, x);
    ys = __fadd_rn(ys, x);
    const float sv = poly ? ys : yc, cv = poly ? yc : ys;
    return make_float2(sign_cos ? -cv : cv, sign_sin ? -sv : sv);
}

__global__ void __launch_bounds__(256) acq_wipeoff_kernel(float2* __restrict__ wipe, uint32_t N, float fs,
    int32_t doppler_max, int32_t doppler_center, int32_t doppler_step, int32_t doppler_bias,
    const float* __restrict__ freqs, int mode)
{
    const uint32_t d = blockIdx.x;
    float2* row = wipe + (size_t)d * N;
    // freqs: the step-two grid (update_grid_doppler_wipeoffs_step2, :307-314)
    const int32_t doppler = -doppler_max + doppler_center + doppler_step * (int32_t)d;
    const float freq = freqs ? freqs[d] : (float)(doppler_bias + doppler);
    if (mode == GSDR_WIPE_EXACT)
        {
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x)
                {
                    const double t = (double)freq * (double)i / (double)fs;
                    double s, c;
                    sincos(-6.283185307179586 * (t - floor(t)), &s, &c);
                    row[i] = make_float2((float)c, (float)s);
                }
            return;
        }
    const float phase_step = __fdiv_rn(__fmul_rn(6.283185307179586f, freq), fs);
    const float inc = -phase_step;
    if (mode == GSDR_WIPE_AVX2)
        {
            const uint32_t iters = N / 8;
            if (threadIdx.x < 8)
                {
                    const uint32_t k = threadIdx.x;
                    float ph = k == 0 ? 0.0f : __fmul_rn((float)k, inc);
                    const float inc8 = __fmul_rn(8.0f, inc);
                    for (uint32_t it = 0; it < iters; ++it)
                        {
                            row[8 * it + k].x = ph;
                            ph = __fadd_rn(ph, inc8);
                        }
                }
            else if (threadIdx.x == 8)
                {
                    float ph = __fmul_rn(inc, (float)(iters * 8));
                    for (uint32_t i = iters * 8; i < N; ++i)
                        {
                            row[i].x = ph;
                            ph = __fadd_rn(ph, inc);
                        }
                }
            __syncthreads();
            for (uint32_t i = threadIdx.x; i < N; i += blockDim.x)
                {
                    if (i < iters * 8)
                        row[i] = cephes_sincos_avx2(row[i].x);
                    else
                        {
                            float s, c;
                            sincosf(row[i].x, &s, &c);
                            row[i] = make_float2(c, s);
                        }
                }
            return;
        }
    if (threadIdx.x == 0)
        {
            float ph = 0.0f;
            for (uint32_t i = 0; i < N; ++i)
                {
                    row[i].x = ph;
                    ph = __fadd_rn(ph, inc);
                }
        }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < N; i += blockDim.x)
        {
            float s, c;
            sincosf(row[i].x, &s, &c);
            row[i] = make_float2(c, s);
        }
}

// ---------------------------------------------------------------- K_code
template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_code_fft_kernel(const float2* __restrict__ codes,
    float2* __restrict__ code_fft, const float2* __restrict__ tw, typename PT::PlanT plan, uint32_t consumed, uint32_t lead)
{
    // set_local_code (pcps_acquisition.cc:176-209): [0 x lead, code[0 .. N - lead)];
    // lead = N - consumed, or N/2 with bit_transition_flag (then only the first N/2
    // code samples of the consumed-long row are used)
    extern __shared__ float2 lds[];
    const uint32_t p = blockIdx.x;
    const float2* c = codes + (size_t)p * consumed;
    float2* out = code_fft + (size_t)p * plan.n;
    const int valid = (int)plan.n - (int)lead;
    auto load = [&](int i) -> float2 {
        int k = i - (int)lead;
        return (k >= 0 && k < valid) ? c[k] : make_float2(0.f, 0.f);
    };
    auto store = [&](int i, float2 v) { out[i] = v; };
    PT::run(plan, lds, tw, load, store);
}

// ---------------------------------------------------------------- K_forward
template <class PT, int IT>
__global__ void __launch_bounds__(PT::NT) acq_forward_kernel(const void* __restrict__ iq, uint64_t block_stride,
    const float2* __restrict__ wipe, float2* __restrict__ X, const float2* __restrict__ tw, typename PT::PlanT plan,
    uint32_t consumed, XMap xm)
{
    extern __shared__ float2 lds[];
    // blockIdx.x = block, blockIdx.y = Doppler bin (of the xm.q stored spectra):
    // the workgroups of one wipe-off row w_d are consecutive, so each XCD's L2
    // fetches the row once per launch (with d fastest every row was re-read from
    // HBM for every block)
    const uint32_t b = blockIdx.x, d = blockIdx.y;
    const size_t base = (size_t)b * block_stride;
    const float2* w = wipe + (size_t)d * plan.n;
    float2* out = X + xm.off(b, d);
    const int ext = (int)(xm.stride - plan.n);  // bins repeated after N - 1 (XMap)
    auto load = [&](int i) -> float2 {
        if (i >= (int)consumed) return make_float2(0.f, 0.f);
        return gsdr::fft::cmul(load_item<IT>(iq, base + i), w[i]);
    };
    auto store = [&](int i, float2 v) {
        out[i] = v;
        if (i < ext) out[plan.n + i] = v;
    };
    PT::run(plan, lds, tw, load, store);
}

// plan types with a packed sub-plan (FourStepPkPlan): the two-launch forward
template <class PT, class = void>
struct requires_subplan : std::false_type
{
};
template <class PT>
struct requires_subplan<PT, std::void_t<typename PT::SubPlan>> : std::true_type
{
};

// ---------------------------------------------------------------- K_forward, two launches (split path)
// The four-step forward transform of the large sizes as two launches instead of one
// workgroup per (b, d) spectrum (320 workgroups at C4 for 256 CUs -- latency-bound):
// acq_forward4_cols_kernel runs the R-point column DFTs of every (b, d) row on
// all CUs (one lane per column, coalesced loads of the wiped-off input, the
// inter-step twiddle W_N^{n2 k1}) into a scratch image of the rows k1 (N2 points
// each, contiguous); acq_forward4_rows_kernel then runs the R * nblocks * D
// sub-transforms on the packed N2-point plan, one per workgroup, storing
// X[k1 + R k2].  The R workgroups of one (b, d) share an XCD, so its L2 merges
// their interleaved output writes.  Same arithmetic as FourStepPkPlan::run.
template <class PT, int IT>
__global__ void __launch_bounds__(256) acq_forward4_cols_kernel(const void* __restrict__ iq, uint64_t block_stride,
    const float2* __restrict__ wipe, float2* __restrict__ scratch, const float2* __restrict__ tw, uint32_t consumed,
    uint32_t D)
{
    using gsdr::pk::c2;
    constexpr int R = PT::R, N2 = PT::N2, N = PT::N;
    const uint32_t row = blockIdx.y;  // b * D + d
    const uint32_t b = row / D, d = row - (row / D) * D;
    const int n2 = (int)(blockIdx.x * 256 + threadIdx.x);
    if (n2 >= N2) return;
    const size_t base = (size_t)b * block_stride;
    const float2* w = wipe + (size_t)d * N;
    c2 v[R];
#pragma unroll
    for (int n1 = 0; n1 < R; ++n1)
        {
            const int i = n1 * N2 + n2;
            v[n1] = i < (int)consumed ? gsdr::pk::from(gsdr::fft::cmul(load_item<IT>(iq, base + i), w[i]))
                                      : c2{0.0f, 0.0f};
        }
    gsdr::pk::Dft<R>::run(v);
    const gsdr::fft::ColTwiddles<R> cw(tw, n2);
    float2* out = scratch + (size_t)row * N;
    out[n2] = gsdr::pk::to(v[0]);
#pragma unroll
    for (int k1 = 1; k1 < R; ++k1) out[(size_t)k1 * N2 + n2] = gsdr::pk::to(gsdr::pk::mul(v[k1], cw(k1)));
}

template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_forward4_rows_kernel(const float2* __restrict__ scratch,
    float2* __restrict__ X, const float2* __restrict__ tw_sub, uint32_t nrows, uint32_t xstride)
{
    using gsdr::pk::c2;
    using SP = typename PT::SubPlan;
    constexpr int R = PT::R, N2 = PT::N2, N = PT::N;
    extern __shared__ float2 lds_raw[];
    // (row, k1), the R workgroups of a row on one XCD (ids dealt round-robin)
    const uint32_t id = blockIdx.x, full = nrows >> 3;
    uint32_t row, k1;
    if (id < full * 8u * R)
        {
            const uint32_t xcd = id & 7u, slot = id >> 3;
            row = (slot / R) * 8u + xcd;
            k1 = slot - (slot / R) * R;
        }
    else
        {
            const uint32_t t = id - full * 8u * R;
            row = full * 8u + t / R;
            k1 = t - (t / R) * R;
        }
    const c2* rk = reinterpret_cast<const c2*>(scratch) + (size_t)row * N + (size_t)k1 * N2;
    // stored spectrum `row` (= b q + d of XMap, d < q) with its E = xstride - N
    // repeated leading bins
    float2* out = X + (size_t)row * xstride;
    const int ext = (int)(xstride - (uint32_t)N);
    auto ld = [&](int, int, int i) -> c2 { return rk[i]; };
    auto st = [&](int k2, c2 v, int) {
        const int k = (int)k1 + R * k2;
        out[k] = gsdr::pk::to(v);
        if (k < ext) out[N + k] = gsdr::pk::to(v);
    };
    SP::template run<false>(reinterpret_cast<c2*>(lds_raw), tw_sub, ld, st, [] {});
}

// ---------------------------------------------------------------- K_correlate
// blockIdx.x = d*P + p (consecutive workgroups share the spectrum X_{b,d}), blockIdx.y = b.
// GRID: also write the full |R|^2 row (the reference's grid dump).
template <class PT, bool GRID>
__global__ void __launch_bounds__(PT::NT) acq_correlate_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, RowStat* __restrict__ stats, float* __restrict__ grid,
    const float2* __restrict__ tw, typename PT::PlanT plan, uint32_t D, uint32_t P, uint32_t prn_slot_for_grid, XMap xm)
{
    extern __shared__ float2 lds[];
    RowStat* scratch = reinterpret_cast<RowStat*>(lds + gsdr::fft::lds_elems_dev(plan));
    const uint32_t N = plan.n;
    uint32_t d, p, b;
    if (GRID)
        {
            d = blockIdx.x;
            p = prn_slot_for_grid;
            b = blockIdx.y;
        }
    else
        {
            // XCD-aware mapping (cdna_hip_programming.md T1): workgroups are dealt
            // round-robin over the 8 XCDs (id % 8), so give all P workgroups of one
            // (b, d) spectrum the same id % 8 — X_{b,d} is then fetched into one
            // XCD's L2 once instead of into all eight.  Speed only, never correctness.
            const uint32_t nrows = gridDim.y * D;  // (b, d) rows
            const uint32_t id = blockIdx.y * gridDim.x + blockIdx.x;
            const uint32_t full = nrows >> 3;     // rows in the XCD-balanced part
            uint32_t row;
            if (id < full * 8u * P)
                {
                    const uint32_t xcd = id & 7u, slot = id >> 3;
                    row = (slot / P) * 8u + xcd;
                    p = slot - (slot / P) * P;
                }
            else
                {
                    const uint32_t t = id - full * 8u * P;  // the last nrows % 8 rows, linear
                    row = full * 8u + t / P;
                    p = t - (t / P) * P;
                }
            b = row / D;
            d = row - b * D;
        }
    const float2* x = X + xm.off(b, d);
    const float2* c = code_fft + (size_t)p * N;
    float best = -1.0f, sum = 0.0f;
    uint32_t bidx = 0xffffffffu;
    // conj(X . conj(C)) = conj(X) . C ; |IFFT(Y)| = |FFT(conj(Y))|
    auto load = [&](int i) -> float2 {
        float2 a = x[i], k = c[i];
        return make_float2(a.x * k.x + a.y * k.y, a.x * k.y - a.y * k.x);
    };
    auto store = [&](int i, float2 v) {
        const float m = v.x * v.x + v.y * v.y;
        if (GRID) grid[(size_t)d * N + i] = m;
        if (stat_better(m, (uint32_t)i, best, bidx))
            {
                best = m;
                bidx = (uint32_t)i;
            }
        sum += m;
    };
    PT::run(plan, lds, tw, load, store);
    if (!GRID)
        {
            block_reduce_stat<PT::NT>(best, bidx, sum, scratch);
            if (threadIdx.x == 0) stats[((size_t)b * P + p) * D + d] = RowStat{best, bidx, sum, 0};
        }
}

// ---------------------------------------------------------------- K_correlate (packed f32)
// The sequential-PRN-group kernel on the packed-f32 FFT (fft_pk.h): one workgroup
// per (row = b*D + d, group of PG PRNs), XCD-aware; the lane's first-stage inputs
// of X_{b,d} stay in VGPRs for the whole group and the next PRN's code-spectrum
// values are fetched by the hook while the current transform runs.  The last
// stage visits each lane's outputs in increasing index order, so a strict '>'
// keeps the lane's first maximum (the reference's index_max semantics).
//
// STAT 1: row (exact max, sum) only -- an order-free reduction, 2.5 VALU per output
//         instead of 7 -- and acq_argmax_pk_kernel recomputes the one row per
//         (b, p) that the grid maximum selects to find its first maximum; the
//         reported peak is then the exact |R|^2, with the reference's first-index
//         rule (32f_index_max_32u) among exact ties.
// STAT 2: row maximum only.  The CFAR statistic needs the sum of one row per
//         (b, p), the row opposite the peak (pcps_acquisition.cc:531-533), so
//         acq_argmax_pk_kernel forms it there by Parseval instead of every row
//         summing its 4000 outputs: sum_n |R[n]|^2 = N sum_k |Y[k]|^2 for the
//         unnormalised transform of Y = conj(X) C.
//
// PG < 0: groups of -PG PRNs without the next-code prefetch (the code values are
// loaded by the first stage itself) -- for plans whose registers cannot hold
// both first-stage operand sets through a transform (N = 16000 on 1024 lanes).
constexpr int pg_count(int pg) { return pg < 0 ? -pg : pg; }

template <class MP, int PG_, int WPE, int STAT>
__global__ void __launch_bounds__(MP::NT) __attribute__((amdgpu_waves_per_eu(WPE))) acq_correlate_pk_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, RowStat* __restrict__ stats, const float2* __restrict__ tw, uint32_t D,
    uint32_t P, uint32_t nblocks, XMap xm)
{
    static_assert(PG_ != 0, "PRN group");
    constexpr int PG = pg_count(PG_);
    constexpr bool PREFETCH = PG_ > 0;
    static_assert(STAT == 1 || STAT == 2, "row statistic 1 (max + sum) or 2 (max)");
    using gsdr::pk::c2;
    constexpr int NT = MP::NT;
    constexpr int NW = NT / 64;
    constexpr int R1 = MP::R1, BPT1 = MP::BPT1, NB1 = MP::NB1;
    constexpr uint32_t N = MP::N;
    extern __shared__ float2 lds_raw[];
    c2* lds = reinterpret_cast<c2*>(lds_raw);
    RowStat* scratch = reinterpret_cast<RowStat*>(lds_raw + MP::lds_bytes() / sizeof(float2));
    const uint32_t G = (P + PG - 1) / PG;
    const uint32_t nrows = nblocks * D;
    const uint32_t id = blockIdx.x;
    const uint32_t full = nrows >> 3;
    uint32_t row, g;
    if (id < full * 8u * G)
        {
            const uint32_t xcd = id & 7u, slot = id >> 3;
            row = (slot / G) * 8u + xcd;
            g = slot - (slot / G) * G;
        }
    else
        {
            const uint32_t t = id - full * 8u * G;
            row = full * 8u + t / G;
            g = t - (t / G) * G;
        }
    const uint32_t b = row / D, d = row - (row / D) * D;
    const uint32_t p0 = g * PG;
    const int np = (int)min((uint32_t)PG, P - p0);
    // the X row and the code spectra through buffer descriptors built from
    // wave-uniform values: per-lane byte offset j*8 in voffset, r*NB1*8 as the
    // scalar/immediate offset -- no 64-bit address arithmetic per load
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(X) + xm.off(b, d), 0, (int)(N * sizeof(c2)), 0x00020000);
    const auto crs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(code_fft) + (size_t)p0 * N, 0, (int)((size_t)np * N * sizeof(c2)), 0x00020000);
    auto bload = [](decltype(xrs) rs, int voff, int soff) -> c2 {
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        return c2{__uint_as_float(u[0]), __uint_as_float(u[1])};
    };
    // a wave with any first-stage butterfly loads for all its lanes (the idle
    // lanes' clamped, in-bounds copies keep every register defined, so no
    // zero-fill code); a wave with none skips the loads
    c2 xr[BPT1][R1], cr[BPT1][R1];
#pragma unroll
    for (int bb = 0; bb < BPT1; ++bb)
        {
            const int j = (int)threadIdx.x + bb * NT;
            const int j0 = (int)(threadIdx.x & ~63u) + bb * NT;
            if (NB1 % NT == 0 || j0 < NB1)
                {
                    const int jj = min(j, NB1 - 1);
#pragma unroll
                    for (int r = 0; r < R1; ++r)
                        {
                            xr[bb][r] = bload(xrs, jj * 8, r * NB1 * 8);
                            if constexpr (PREFETCH) cr[bb][r] = bload(crs, jj * 8, r * NB1 * 8);
                        }
                }
        }
    for (int q = 0; q < np; ++q)
        {
            {
                    float rmax = 0.0f, sum = 0.0f;
                    auto load = [&](int bb, int r, int i) -> c2 {
                        if constexpr (PREFETCH)
                            return gsdr::pk::conj_mul(xr[bb][r], cr[bb][r]);
                        else
                            return gsdr::pk::conj_mul(xr[bb][r], bload(crs, i * 8, (int)(q * N * 8)));
                    };
                    auto hook = [&]() {
                        if (PREFETCH && q + 1 < np)
                            {
#pragma unroll
                                for (int bb = 0; bb < BPT1; ++bb)
                                    {
                                        const int j = (int)threadIdx.x + bb * NT;
                                        if (NB1 % NT == 0 || j < NB1)
                                            {
#pragma unroll
                                                for (int r = 0; r < R1; ++r)
                                                    cr[bb][r] = bload(crs, j * 8, (int)((q + 1) * N * 8) + r * NB1 * 8);
                                            }
                                    }
                            }
                    };
                    auto store = [&](int, c2 v, int) {
                        const float m = __builtin_fmaf(v.x, v.x, v.y * v.y);
                        rmax = __builtin_fmaxf(rmax, m);
                        if constexpr (STAT == 1) sum += m;
                    };
                    MP::template run<false>(lds, tw, load, store, hook);
                    rmax = gsdr::wave_max(rmax);
                    if constexpr (STAT == 1)
                        {
#pragma unroll
                            for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
                        }
                    RowStat* sc = scratch + (q & 1) * NW;
                    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
                    if (lane == 0) sc[wave] = RowStat{rmax, 0u, sum, 0};
                    __syncthreads();
                    if (threadIdx.x == 0)
                        {
                            RowStat best = sc[0];
#pragma unroll
                            for (int w = 1; w < NW; ++w)
                                {
                                    best.max = __builtin_fmaxf(best.max, sc[w].max);
                                    best.sum += sc[w].sum;
                                }
                            stats[((size_t)b * P + p0 + q) * D + d] = best;
                        }
            }
        }
}

// ---------------------------------------------------------------- K_correlate, register four-step
// For transforms whose full LDS image allows only one workgroup per CU (N = 16000
// at 16 Msps: 128 KB, so the workgroup's barriers and first-stage loads cannot
// overlap another's work).  N = R * L, decimation in frequency as in fft_4step.h:
//   phase 1: every lane takes CPL columns n2 of the R x L view, loads the R products
//            conj(X[n1 L + n2]) C[n1 L + n2] (coalesced), runs the packed DFT_R and
//            scales row k1 by W_N^{n2 k1} -- the whole transform now sits in VGPRs
//            (R * CPL complex per lane);
//   phase 2: R/H rounds: H rows go to LDS (H * L complex -- 64 KB for H = 8, L =
//            1000, so two workgroups share a CU), H batched L-point Stockham
//            transforms run there, the last stage's |.|^2 feeds the row maximum.
// Only the row maximum is kept (STAT 2): the outputs arrive in no particular order
// and duplicated (clamped) lanes only repeat values, which a maximum ignores.
// acq_argmax_pk_kernel recomputes the selected row on the full-LDS plan for the
// first-maximum index and the exact peak.
// Row layouts in LDS: row rw at rw * stride, element e at e + (e / S) * P -- one
// pad of P elements every S, so strided Stockham writes could spread over the banks.
// The stage functions need S | Ns (writes) and S | L/R (reads) so every address
// is a per-butterfly base plus a compile-time offset.  Pads chosen with an LDS bank
// model halved the measured bank conflicts of the 1000-point rows (0.30 -> 0.15 of
// the LDS-active cycles) and left the time unchanged -- the rows are VALU-issue bound
// (profiles/r05p) -- so every plan runs unpadded (NoPads).
template <int L, int S, int P>
struct RowPad
{
    static constexpr int stride = L + (S ? (L / S) * P : 0);
    static constexpr int pad_every = S;
    __device__ __forceinline__ static int pad(int e) { return S ? e + (e / S) * P : e; }
    static constexpr int cpad(int e) { return S ? e + (e / S) * P : e; }
};

template <int R, int NT, int L, int H, int Ns, bool LAST, class In, class OutL, class Out>
__device__ __forceinline__ void rows_stage(gsdr::pk::c2* lds, Out& out, int row0)
{
    using gsdr::pk::c2;
    constexpr int NB = L / R;       // butterflies per row
    constexpr int TOT = H * NB;     // butterflies of the stage
    constexpr int BPT = (TOT + NT - 1) / NT;
    constexpr int TSTRIDE = L / (Ns * R);
    // reads: element jb + r NB, pad(jb) + cpad(r NB) needs S | NB
    static_assert(In::pad_every == 0 || NB % In::pad_every == 0, "read layout: S must divide L/R");
    // writes: element (jb - k) R + k + r Ns (k < Ns), pad((jb - k) R) + k + cpad(r Ns)
    // needs S | Ns R and Ns | S
    static_assert(LAST || OutL::pad_every == 0 || ((Ns * R) % OutL::pad_every == 0 && OutL::pad_every % Ns == 0),
        "write layout: S must divide Ns R and be a multiple of Ns");
    const int wbase = (int)(threadIdx.x & ~63u);
    c2 v[BPT][R];
    int jb[BPT], rw[BPT];
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            const int jj = min((int)threadIdx.x + b * NT, TOT - 1);
            rw[b] = jj / NB;
            jb[b] = jj - rw[b] * NB;
            if (TOT % NT == 0 || wbase + b * NT < TOT)
                {
                    // element jb + r NB: the pad of r NB is compile-time (S | NB)
                    const int base = rw[b] * In::stride + In::pad(jb[b]);
#pragma unroll
                    for (int r = 0; r < R; ++r) v[b][r] = lds[base + In::cpad(r * NB)];
                }
        }
    __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            if (TOT % NT == 0 || wbase + b * NT < TOT)
                {
                    int k = 0;
                    if constexpr (Ns > 1)
                        {
                            k = jb[b] % Ns;
                            gsdr::pk::apply_powers<R>(v[b], gsdr::pk::from(out.twiddle(k * TSTRIDE)));
                        }
                    gsdr::pk::Dft<R>::run(v[b]);
                    if constexpr (LAST)
                        {
#pragma unroll
                            for (int r = 0; r < R; ++r) out.value(v[b][r], jb[b] + r * Ns, row0 + rw[b]);  // row output jb + r Ns
                        }
                    else
                        {
                            // element (jb - k) R + k + r Ns: with S | Ns and S | Ns R the
                            // pad splits into the butterfly's part and a compile-time r part
                            const int base = rw[b] * OutL::stride + OutL::pad((jb[b] - k) * R) + k;
#pragma unroll
                            for (int r = 0; r < R; ++r) lds[base + OutL::cpad(r * Ns)] = v[b][r];
                        }
                }
        }
    if constexpr (!LAST) __syncthreads();
}

template <int NT, int L, int H, int Ns, class Pads, int Si, int R, int... Rest, class Out>
__device__ __forceinline__ void rows_stages(gsdr::pk::c2* lds, Out& out, int row0)
{
    constexpr bool LAST = sizeof...(Rest) == 0;
    using In = typename Pads::template layout<Si>;
    using OutL = typename Pads::template layout<LAST ? Si : Si + 1>;
    rows_stage<R, NT, L, H, Ns, LAST, In, OutL>(lds, out, row0);
    if constexpr (!LAST) rows_stages<NT, L, H, Ns * R, Pads, Si + 1, Rest...>(lds, out, row0);
}

// Pads for the buffers between the row stages (buffer 0 = phase 1's rows); a
// bank-model padding of the 1000-point rows measured within noise.
template <int L>
struct NoPads
{
    template <int I>
    using layout = RowPad<L, 0, 0>;
};

// ---- wave-local row transforms
// One wave transforms one L-point row in place in its own LDS row buffer: the
// Stockham exchange between the row stages needs no workgroup barrier, because
// a wave's LDS instructions execute in issue order -- every lane's reads of a
// stage are issued before any of its writes, and the next stage's reads after
// them.  The empty asm statements (memory clobber) keep the compiler from moving
// a write above a read whose address it believes distinct (other lanes' data is
// involved, which per-thread alias analysis cannot see).  Lanes past the stage's
// butterfly count repeat the last butterfly (same values to the same addresses,
// repeated outputs for an order-free maximum), so no lane is predicated off.
template <int R, int L, int Ns, bool LAST, class In, class OutL, class Out>
__device__ __forceinline__ void wl_stage(gsdr::pk::c2* row, Out& out, int lane, int k1)
{
    using gsdr::pk::c2;
    constexpr int NB = L / R;
    constexpr int BPT = (NB + 63) / 64;
    constexpr int TSTRIDE = L / (Ns * R);
    static_assert(In::pad_every == 0 || NB % In::pad_every == 0, "read layout: S must divide L/R");
    static_assert(LAST || OutL::pad_every == 0 || ((Ns * R) % OutL::pad_every == 0 && OutL::pad_every % Ns == 0),
        "write layout: S must divide Ns R and be a multiple of Ns");
    c2 v[BPT][R];
    int jb[BPT];
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            jb[b] = NB % 64 == 0 ? lane + 64 * b : min(lane + 64 * b, NB - 1);
            const int base = In::pad(jb[b]);
#pragma unroll
            for (int r = 0; r < R; ++r) v[b][r] = row[base + In::cpad(r * NB)];
        }
    asm volatile("" ::: "memory");
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            int k = 0;
            if constexpr (Ns > 1)
                {
                    k = jb[b] % Ns;
                    gsdr::pk::apply_powers<R>(v[b], gsdr::pk::from(out.twiddle(k * TSTRIDE)));
                }
            gsdr::pk::Dft<R>::run(v[b]);
            if constexpr (LAST)
                {
#pragma unroll
                    for (int r = 0; r < R; ++r) out.value(v[b][r], jb[b] + r * Ns, k1);
                }
            else
                {
                    const int base = OutL::pad((jb[b] - k) * R) + k;
#pragma unroll
                    for (int r = 0; r < R; ++r) row[base + OutL::cpad(r * Ns)] = v[b][r];
                }
        }
    if constexpr (!LAST) asm volatile("" ::: "memory");
}

template <int L, int Ns, class Pads, int Si, int R, int... Rest, class Out>
__device__ __forceinline__ void wl_stages(gsdr::pk::c2* row, Out& out, int lane, int k1)
{
    constexpr bool LAST = sizeof...(Rest) == 0;
    using In = typename Pads::template layout<Si>;
    using OutL = typename Pads::template layout<LAST ? Si : Si + 1>;
    wl_stage<R, L, Ns, LAST, In, OutL>(row, out, lane, k1);
    if constexpr (!LAST) wl_stages<L, Ns * R, Pads, Si + 1, Rest...>(row, out, lane, k1);
}

// WPE_ packs the waves-per-EU hint (bits 0-3) and PGS (bits 4+): with PGS > 0 an
// XCD walks its rows PRN-group-major (groups of PGS PRNs, PGS | P), so its L2 holds
// PGS code spectra (PGS x 128 KB at N = 16000) instead of cycling through all P.
// H_ = 0: wave-local rows (WL): each round puts one row per wave in LDS and every
// wave transforms its own row without workgroup barriers (wl_stages); H = NT / 64
// rows per round, the last round partial when NT / 64 does not divide R.
template <int R_, int NT_, int H_, int WPE_, class Pads_, int... Rs>
struct RegFourStep
{
    static constexpr bool WL = H_ == 0;
    static constexpr int R = R_, NT = NT_, H = WL ? NT_ / 64 : H_, WPE = WPE_ & 15, PGS = WPE_ >> 4;
    static constexpr int L = (Rs * ...);
    static constexpr int N = R * L;
    static constexpr int CPL = (L + NT - 1) / NT;
    using Pads = Pads_;
    static constexpr int max_stride()
    {
        int m = L;
        constexpr int ns = sizeof...(Rs);
        if (ns > 1 && Pads::template layout<1>::stride > m) m = Pads::template layout<1>::stride;
        if (ns > 2 && Pads::template layout<2>::stride > m) m = Pads::template layout<2>::stride;
        if (ns > 3 && Pads::template layout<3>::stride > m) m = Pads::template layout<3>::stride;
        return m;
    }
    static constexpr int lds_elems = H * max_stride();
    static constexpr size_t lds_bytes() { return (size_t)lds_elems * sizeof(float2) + (NT / 64) * sizeof(float); }
    template <class Out>
    __device__ __forceinline__ static void row_transforms(gsdr::pk::c2* lds, Out& out, int row0)
    {
        rows_stages<NT, L, H, 1, Pads, 0, Rs...>(lds, out, row0);
    }
    // WL: one row (at lds, max_stride() elements) by the calling wave
    template <class Out>
    __device__ __forceinline__ static void wl_row(gsdr::pk::c2* row, Out& out, int lane, int k1)
    {
        wl_stages<L, 1, Pads, 0, Rs...>(row, out, lane, k1);
    }

    // Phase 2 of T register four-steps at once (LDS rounds of H rows): rows g = j R + k1
    // of transform j, so a round may hold rows of two transforms; out.value receives g
    // as the row index.  A last round with fewer than H rows leaves the rest of the LDS
    // rows stale: their outputs carry g >= T R, which out.value must drop.
    template <int T, int CPL, class Out>
    __device__ __forceinline__ static void phase2_multi(gsdr::pk::c2* lds, gsdr::pk::c2 (&v)[T][CPL][R], Out& out)
    {
        static_assert(!WL, "multi-transform phase 2: LDS rounds of H rows");
        const int wbase = (int)(threadIdx.x & ~63u);
#pragma unroll
        for (int h = 0; h < (T * R + H - 1) / H; ++h)
            {
                if (h > 0) __syncthreads();  // the previous round's last-stage reads are done
#pragma unroll
                for (int c = 0; c < CPL; ++c)
                    {
                        const int n2 = min((int)threadIdx.x + c * NT, L - 1);
                        if (L % NT == 0 || wbase + c * NT < L)
                            {
#pragma unroll
                                for (int i = 0; i < H; ++i)
                                    if (h * H + i < T * R) lds[i * L + n2] = v[(h * H + i) / R][c][(h * H + i) % R];
                            }
                    }
                __syncthreads();
                row_transforms(lds, out, h * H);
            }
    }
    // Phase 2 of a register four-step: the R rows (phase 1's v[c][k1], lane column
    // n2 = threadIdx.x + c NT, clamped) through LDS and the L-point row transforms.
    template <int CPL, class Out>
    __device__ __forceinline__ static void phase2(gsdr::pk::c2* lds, gsdr::pk::c2 (&v)[CPL][R], Out& out)
    {
        const int wbase = (int)(threadIdx.x & ~63u);
        auto column = [&](int c, int& n2) -> bool {
            n2 = min((int)threadIdx.x + c * NT, L - 1);
            return L % NT == 0 || wbase + c * NT < L;
        };
        if constexpr (!WL)
            {
                static_assert(R % H == 0, "rows go through LDS in groups of H");
#pragma unroll
                for (int h = 0; h < R / H; ++h)
                    {
                        if (h > 0) __syncthreads();  // the previous group's last-stage reads are done
#pragma unroll
                        for (int c = 0; c < CPL; ++c)
                            {
                                int n2;
                                if (column(c, n2))
                                    {
#pragma unroll
                                        for (int i = 0; i < H; ++i) lds[i * L + n2] = v[c][h * H + i];
                                    }
                            }
                        __syncthreads();
                        row_transforms(lds, out, h * H);
                    }
            }
        else
            {
                using L0 = typename Pads::template layout<0>;
                constexpr int STR = max_stride();
                const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
#pragma unroll
                for (int h = 0; h < (R + H - 1) / H; ++h)
                    {
                        if (h > 0) __syncthreads();  // every wave's row of the previous round is done
#pragma unroll
                        for (int c = 0; c < CPL; ++c)
                            {
                                int n2;
                                if (column(c, n2))
                                    {
#pragma unroll
                                        for (int i = 0; i < H; ++i)
                                            if (h * H + i < R) lds[i * STR + L0::pad(n2)] = v[c][h * H + i];
                                    }
                            }
                        __syncthreads();
                        if (h * H + wave < R) wl_row(lds + wave * STR, out, lane, h * H + wave);
                    }
            }
    }
};

template <class RP>
__global__ void __launch_bounds__(RP::NT) __attribute__((amdgpu_waves_per_eu(RP::WPE))) acq_correlate_reg_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, RowStat* __restrict__ stats, const float2* __restrict__ tw, uint32_t D,
    uint32_t P, uint32_t nblocks, XMap xm)
{
    using gsdr::pk::c2;
    constexpr int R = RP::R, NT = RP::NT, L = RP::L, CPL = RP::CPL;
    constexpr uint32_t N = RP::N;
    constexpr int NW = NT / 64;
    extern __shared__ float2 lds_raw[];
    c2* lds = reinterpret_cast<c2*>(lds_raw);
    float* red = reinterpret_cast<float*>(lds_raw + RP::lds_elems);
    // (row = b*D + d, PRN p), XCD-aware: the P workgroups of one row on one XCD
    const uint32_t nrows = nblocks * D;
    const uint32_t id = blockIdx.x;
    const uint32_t full = nrows >> 3;
    uint32_t row, p;
    if (id < full * 8u * P)
        {
            const uint32_t xcd = id & 7u, slot = id >> 3;
            if (RP::PGS > 0 && P % (uint32_t)RP::PGS == 0)
                {
                    const uint32_t per_group = full * (uint32_t)RP::PGS;
                    const uint32_t pg = slot / per_group, rem = slot - pg * per_group;
                    const uint32_t ri = rem / (uint32_t)RP::PGS;
                    row = ri * 8u + xcd;
                    p = pg * (uint32_t)RP::PGS + (rem - ri * (uint32_t)RP::PGS);
                }
            else
                {
                    row = (slot / P) * 8u + xcd;
                    p = slot - (slot / P) * P;
                }
        }
    else
        {
            const uint32_t t = id - full * 8u * P;
            row = full * 8u + t / P;
            p = t - (t / P) * P;
        }
    const uint32_t b = row / D, d = row - (row / D) * D;
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(X) + xm.off(b, d), 0, (int)(N * sizeof(c2)), 0x00020000);
    const auto crs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(code_fft) + (size_t)p * N, 0, (int)(N * sizeof(c2)), 0x00020000);
    auto bload = [](decltype(xrs) rs, int voff, int soff) -> c2 {
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        return c2{__uint_as_float(u[0]), __uint_as_float(u[1])};
    };
    const int wbase = (int)(threadIdx.x & ~63u);
    // phase 1: columns (clamped: a lane past L repeats column L-1, whose values
    // are written to the same LDS words and only repeat outputs)
    c2 v[CPL][R];
#pragma unroll
    for (int c = 0; c < CPL; ++c)
        {
            if (L % NT == 0 || wbase + c * NT < L)
                {
                    const int n2 = min((int)threadIdx.x + c * NT, L - 1);
#pragma unroll
                    for (int n1 = 0; n1 < R; ++n1)
                        v[c][n1] = gsdr::pk::conj_mul(bload(xrs, n2 * 8, n1 * L * 8), bload(crs, n2 * 8, n1 * L * 8));
                    gsdr::pk::Dft<R>::run(v[c]);
                    gsdr::pk::apply_powers<R>(v[c], gsdr::pk::from(tw[n2]));
                }
        }
    struct Out
    {
        const float2* tw;
        float m;
        __device__ __forceinline__ float2 twiddle(int m_) const { return tw[m_ * R]; }  // W_L^m = W_N^{m R}
        __device__ __forceinline__ void value(c2 x, int, int) { m = __builtin_fmaxf(m, __builtin_fmaf(x.x, x.x, x.y * x.y)); }
    } out{tw, 0.0f};
    // phase 2: the rows k1 through LDS
    RP::phase2(lds, v, out);
    float rmax = gsdr::wave_max(out.m);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) red[wave] = rmax;
    __syncthreads();
    if (threadIdx.x == 0)
        {
            float best = red[0];
#pragma unroll
            for (int w2 = 1; w2 < NW; ++w2) best = __builtin_fmaxf(best, red[w2]);
            stats[((size_t)b * P + p) * D + d] = RowStat{best, 0u, 0.0f, 0};
        }
}

// ---------------------------------------------------------------- K_correlate, split register four-step (large N)
// Transforms too large for one workgroup's registers (N = 64000: 512 KB, the whole
// register file of a CU; N = 100000) and the register-resident ones beyond the
// LDS engine (N = 25000, 32000).  Outer decimation in frequency by ROUT:
//   X[q + ROUT k'] = sum_m W_M^{m k'} z_q[m],   m < M = N / ROUT,
//   z_q[m] = W_N^{m q} sum_{r < ROUT} Y[r M + m] W_ROUT^{r q},
// so the ROUT sub-transforms own disjoint output sets and each one is a workgroup
// of its own: an M-point register four-step (phase 1 columns in VGPRs, phase 2
// rows through LDS, RegFourStep RP) whose loads form z_q from the ROUT products
// Y = conj(X) C of its input positions.  Nothing round-trips through a global
// scratch row (the packed four-step's phase-1 rows did, 2 x 8 N bytes per
// transform); a sub-transform re-reads the whole X and code rows instead, which
// the XCD-aware walk below keeps in L2.  Only the row maximum is kept (STAT 2,
// atomically merged over the ROUT sub-transforms); acq_argmax_four_kernel
// recomputes the selected row for the first-maximum index and the CFAR power.
// HALF (bit_transition_flag): only outputs k >= N / 2 are the reference's
// effective window (pcps_acquisition.cc:671); with k = q + ROUT (k1 + R k2),
// k >= N / 2 exactly when the row output k2 >= L / 2.
// Grid: one workgroup per (row = b*D + d, PRN p, sub-transform q), the ROUT*P
// workgroups of one row on one XCD, each XCD walking its rows in groups of pgs
// PRNs so its L2 holds pgs code rows while the X rows stream.
// ARG: the selected row's pass instead of the grid (acq_reduce_kernel chose Doppler
// row d* of (b, p) from the row maxima): grid (b*P + p, q), the same arithmetic as
// the grid pass (the recomputed values are bit-identical to those the row maximum
// came from), each output's key (|R|^2 bits, ~j) merged into keys[b*P + p] by a
// 64-bit atomic maximum -- the first maximum over the effective window j = k -
// (N - eff), index_max's rule (KERN/32f_index_max_32u.h:446-467) -- and, for the
// peak ratio, |R|^2 into the row's rowbuf entries; acq_argmax_split_finish_kernel
// turns the key into the result fields.  One workgroup per transform of a
// 100000-point row spreads the pass over ROUT x more CUs than the one-workgroup
// recomputation (acq_argmax_four_kernel: 144 workgroups at C5 Galileo).
// The input factor W_N^{m q} of sub-transform q is a compile-time root per column row
// and one table read per column (r04e: C4 bit transition +11 % over R reads).
// phase 1 staged through per-wave LDS rings (split_staged): the copies in flight per
// wave (2 KB of LDS each); 0: products straight from VGPR loads everywhere
#ifndef GSDR_SPLIT_DMA
#define GSDR_SPLIT_DMA 4
#endif
// the smallest outer radix staged (1: the 512-lane 25000 plan too), besides the
// one-column-per-lane plans, which are staged at any outer radix
#ifndef GSDR_SPLIT_DMA_MIN_ROUT
#define GSDR_SPLIT_DMA_MIN_ROUT 2
#endif
// waves per SIMD the staged grid pass is compiled for (4: <= 128 VGPRs, two 512-lane
// workgroups per CU as the VGPR form had)
#ifndef GSDR_SPLIT_WPE
#define GSDR_SPLIT_WPE 4
#endif
// staged phase 1's per-wave ring: slots of one X and PPW code copies (1 KB each per
// wave), as many in flight as GSDR_SPLIT_DMA allows within 144 KB per workgroup
template <class RP, int PPW>
struct SplitRing
{
    static constexpr int slot = 1024 * (1 + PPW);
    static constexpr int fit = 147456 / ((RP::NT / 64) * slot);
    static constexpr int depth = GSDR_SPLIT_DMA < fit ? GSDR_SPLIT_DMA : (fit > 0 ? fit : 1);
    static constexpr size_t bytes = (size_t)(RP::NT / 64) * depth * slot;
};

// which split plans stage phase 1 (r06, profiles/r06b3: 100000 = 4 x 25000 118 -> 133
// Msps, 64000 = 2 x 32000 88 -> 98, 32000 (one column per lane on 1024 lanes) 105 ->
// 118; the 512-lane 25000 plan, whose loads already go out 50 per column at once,
// 143 -> 138: left on VGPR loads)
template <int ROUT, class RP>
constexpr bool split_staged()
{
    return GSDR_SPLIT_DMA > 0 && (ROUT >= GSDR_SPLIT_DMA_MIN_ROUT || RP::CPL == 1);
}

// dynamic LDS of a split launch: phase 2's rows (+ the reduction slots) or, staged,
// each wave's ring of GSDR_SPLIT_DMA 2 KB copy slots, whichever is larger
template <int ROUT, class RP, int PPW = 1>
constexpr size_t split_lds_bytes()
{
    constexpr size_t ring = split_staged<ROUT, RP>() ? SplitRing<RP, PPW>::bytes : 0;
    return ring > RP::lds_bytes() ? ring : RP::lds_bytes();
}

template <int ROUT, class RP, bool HALF, bool ARG = false, int QPW = 1, int PPW = 1>
__global__ void __launch_bounds__(RP::NT) __attribute__((amdgpu_waves_per_eu(
    ARG ? 1 : (split_staged<ROUT, RP>() ? GSDR_SPLIT_WPE : RP::WPE)))) acq_correlate_split_kernel(
    const float2* __restrict__ X, const float2* __restrict__ code_fft, RowStat* __restrict__ stats,
    const float2* __restrict__ tw, uint32_t D, uint32_t P, uint32_t nblocks, uint32_t pgs, XMap xm,
    const gsdr_acq_result* __restrict__ sel, unsigned long long* __restrict__ keys, float* __restrict__ rowbuf,
    float* __restrict__ psum)
{
    using gsdr::pk::c2;
    constexpr int R = RP::R, NT = RP::NT, L = RP::L, CPL = RP::CPL;
    constexpr uint32_t M = RP::N;
    constexpr uint32_t N = M * ROUT;
    constexpr int NW = NT / 64;
    extern __shared__ float2 lds_raw[];
    c2* lds = reinterpret_cast<c2*>(lds_raw);
    float* red = reinterpret_cast<float*>(lds_raw + RP::lds_elems);
    // QPW sub-transforms per workgroup: q = qq + j RQ (j < QPW) -- they share every
    // product Y[r M + m] (only the exact outer factors W_ROUT^{r q} differ)
    static_assert(ROUT % QPW == 0 && (QPW == 1 || split_staged<ROUT, RP>()), "sub-transforms per workgroup");
    // or PPW PRNs per workgroup (ROUT 1): transform j correlates PRN p + j against the
    // same X row, read once for all of them
    static_assert(PPW == 1 || (ROUT == 1 && QPW == 1 && !ARG && PPW == 2 && split_staged<ROUT, RP>()),
        "PRNs per workgroup");
    constexpr int T = QPW * PPW;  // transforms per workgroup
    constexpr int RQ = ROUT / QPW;
    const uint32_t PV = P / PPW * RQ;  // virtual PRNs: pv = (p / PPW) RQ + qq
    const uint32_t nrows = nblocks * D;
    const uint32_t id = blockIdx.x;
    const uint32_t full = nrows >> 3;
    uint32_t row, pv;
    if constexpr (ARG)
        {
            const uint32_t bp = id / RQ;
            const uint32_t dsel = sel[bp].doppler_index;
            if (dsel >= D) return;  // uniform: no maximum found (an all-NaN grid)
            row = (bp / P) * D + dsel;
            pv = (bp - (bp / P) * P) * RQ + (id - bp * RQ);
        }
    else if (id < full * 8u * PV)
        {
            const uint32_t xcd = id & 7u, slot = id >> 3;
            const uint32_t G = pgs * RQ;  // PV % G == 0 (host)
            const uint32_t per_group = full * G;
            const uint32_t pg = slot / per_group, rem = slot - pg * per_group;
            const uint32_t ri = rem / G;
            row = ri * 8u + xcd;
            pv = pg * G + (rem - ri * G);
        }
    else
        {
            const uint32_t t = id - full * 8u * PV;
            row = full * 8u + t / PV;
            pv = t - (t / PV) * PV;
        }
    const uint32_t p = pv / RQ * PPW, q = pv - pv / RQ * RQ;  // q: the first sub-transform (qq); p the first PRN
    const uint32_t b = row / D, d = row - (row / D) * D;
    const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float2*>(X) + xm.off(b, d), 0, (int)(N * sizeof(c2)),
        0x00020000);
    const auto crs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float2*>(code_fft) + (size_t)p * N, 0, (int)(N * PPW * sizeof(c2)), 0x00020000);
    auto bload = [](decltype(xrs) rs, int voff, int soff) -> c2 {
        const auto u = __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0);
        return c2{__uint_as_float(u[0]), __uint_as_float(u[1])};
    };
    const float2* xg = X + xm.off(b, d);
    const float2* cg = code_fft + (size_t)p * N;
    (void)xg;
    (void)cg;
    static_assert(ROUT == 1 || ROUT == 2 || ROUT == 4, "outer radix 1, 2 or 4");
    const int wbase = (int)(threadIdx.x & ~63u);
    // phase 1: columns (clamped lanes repeat column L-1), with the sub-transform
    // index q a compile-time constant: the outer factors W_ROUT^{rq} are exact
    // (+-1, +-i: an add/sub with swapped operands) and W_N^{mq} one table read
    // (m q < N)
    c2 v[T][CPL][R];
    // ROUT > 1: every element of a column sums ROUT products.  Loaded into VGPRs,
    // the compiler kept the accumulated columns resident and issued two loads and a
    // wait per product (r05: 200 dependent L2 round trips per column at 100000, VALU
    // issuing 29 % of the cycles).  Staged instead: each wave copies its own
    // columns' X and code values into its own LDS ring with global_load_lds
    // (dwordx4: one instruction moves two 512-byte segments -- one (row n1, quarter r,
    // column set c) each -- without VGPRs), DEPTH copies ahead of the products that
    // read them; no other wave reads a wave's ring, so no barrier, only its vmcnt.
    // Each element's sum keeps the r order (bit-identical).
    auto phase1_dma = [&](auto qc) {
        constexpr int Q = decltype(qc)::value;
        constexpr int DEPTH = SplitRing<RP, PPW>::depth, SLOT = SplitRing<RP, PPW>::slot;
        // segment s: column set c = s / U, unit u = s % U (n1 = u / ROUT, r = u % ROUT):
        // column-major, so a column's transform runs (and its registers settle) before
        // the next column accumulates, as in the VGPR form
        constexpr int U = R * ROUT;
        constexpr int PPC = (U + 1) / 2;          // copy pairs per column set (an odd U repeats its last unit)
        constexpr int PAIRS = PPC * CPL;         // one X and one code copy per two segments
        const int wave = (int)(threadIdx.x >> 6), lane = (int)(threadIdx.x & 63);
        char* ring = reinterpret_cast<char*>(lds_raw) + (size_t)wave * DEPTH * SLOT;
        const int half = lane >> 5, l32 = lane & 31;
        const int lane_off = (wave * 64 + 2 * l32) * 8;
        auto issue = [&](auto kc) {
            constexpr int k = decltype(kc)::value;
            if constexpr (k < PAIRS)
                {
                    // lanes 0-31: unit 2kk of column set c, lanes 32-63: unit 2kk + 1 (an odd
                    // unit count repeats its last); two columns (16 B) per lane
                    constexpr int c = k / PPC, kk = k % PPC;
                    constexpr int ua = 2 * kk, ub = 2 * kk + 1 < U ? 2 * kk + 1 : 2 * kk;
                    constexpr int ea = (ua % ROUT) * (int)M + (ua / ROUT) * L + c * NT;
                    constexpr int eb = (ub % ROUT) * (int)M + (ub / ROUT) * L + c * NT;
                    // this lane's 16 bytes: the lane part in voffset, the first segment's
                    // element offset as the (uniform) scalar offset; bounds-checked buffer
                    // copies (lanes past column L - 1 copy bytes no lane reads, past the
                    // row's end zeros)
                    const int voff = lane_off + half * ((eb - ea) * 8);
                    char* dst = ring + (k % DEPTH) * SLOT;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(xrs, (gsdr_lvoid*)dst, 16, voff, ea * 8, 0, 0);
#pragma unroll
                    for (int j = 0; j < PPW; ++j)
                        __builtin_amdgcn_raw_ptr_buffer_load_lds(crs, (gsdr_lvoid*)(dst + 1024 * (1 + j)), 16, voff,
                            (ea + j * (int)N) * 8, 0, 0);
                }
        };
        // the lane's column within its segment (clamped lanes read column L - 1's)
        int cl[CPL];
#pragma unroll
        for (int c = 0; c < CPL; ++c) cl[c] = min((int)threadIdx.x + c * NT, L - 1) - (c * NT + wave * 64);
        auto prologue = [&](auto kc) { issue(kc); };
        gsdr::pk::static_for<0, DEPTH>(prologue);
        auto step = [&](auto kc) {
            constexpr int k = decltype(kc)::value;
            // pair k has landed once at most (1 + PPW) (min(DEPTH, PAIRS - k) - 1) younger copies are out
            constexpr int younger = (1 + PPW) * ((PAIRS - k < DEPTH ? PAIRS - k : DEPTH) - 1);
            // s_waitcnt vmcnt(younger) (expcnt / lgkmcnt left at their maxima)
            __builtin_amdgcn_s_waitcnt((younger & 15) | (7 << 4) | (15 << 8) | ((younger >> 4) << 14));
            const char* src = ring + (k % DEPTH) * SLOT;
            auto seg = [&](auto jc) {
                constexpr int c = k / PPC, u = 2 * (k % PPC) + decltype(jc)::value;
                if constexpr (u < U)
                    {
                        constexpr int n1 = u / ROUT, r = u % ROUT;
                        if (L % NT == 0 || wbase + c * NT < L)
                            {
                                const int off = decltype(jc)::value * 512 + cl[c] * 8;
                                const c2 xv = *reinterpret_cast<const c2*>(src + off);
                                const c2 cv = *reinterpret_cast<const c2*>(src + 1024 + off);
                                const c2 y = gsdr::pk::conj_mul(xv, cv);
                                auto acc = [&](auto jq) {
                                    constexpr int J = decltype(jq)::value;
                                    constexpr int QJ = Q + (PPW == 1 ? J * RQ : 0);
                                    // W_ROUT^{r QJ} = W_4^{e}, e = (r QJ mod ROUT) * 4 / ROUT
                                    constexpr int e = ((r * QJ) % ROUT) * (4 / ROUT);
                                    c2& z = v[J][c][n1];
                                    if constexpr (PPW > 1 && J > 0)
                                        z = gsdr::pk::conj_mul(xv, *reinterpret_cast<const c2*>(src + 1024 * (1 + J) + off));
                                    else if constexpr (r == 0)
                                        z = y;
                                    else if constexpr (e == 0)
                                        z = z + y;
                                    else if constexpr (e == 1)
                                        z = gsdr::pk::add_mi(z, y);  // z + (-i) y
                                    else if constexpr (e == 2)
                                        z = z - y;
                                    else
                                        z = gsdr::pk::sub_mi(z, y);  // z + i y
                                    if constexpr (QJ > 0 && r == ROUT - 1) z = gsdr::pk::mul_root<QJ * n1, ROUT * R>(z);
                                };
                                gsdr::pk::static_for<0, T>(acc);
                            }
                    }
            };
            gsdr::pk::static_for<0, 2>(seg);
            // the slot's reads are done (their values are used above): refill it
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            issue(std::integral_constant<int, k + DEPTH>{});
            // a column's last pair: its transform, while the next column's copies land
            // (fenced: interleaved with the next column's sums it spilled)
            if constexpr ((k + 1) % PPC == 0)
                {
                    constexpr int c = k / PPC;
                    __builtin_amdgcn_sched_barrier(0);
                    if (L % NT == 0 || wbase + c * NT < L)
                        {
                            const int n2 = min((int)threadIdx.x + c * NT, L - 1);
                            auto transform = [&](auto jq) {
                                constexpr int QJ = Q + (PPW == 1 ? decltype(jq)::value * RQ : 0);
                                c2(&w)[R] = v[decltype(jq)::value][c];
                                gsdr::pk::Dft<R>::run(w);
                                if constexpr (QJ > 0)
                                    {
                                        const c2 w0 = gsdr::pk::from(tw[QJ * n2]);
#pragma unroll
                                        for (int k1 = 0; k1 < R; ++k1) w[k1] = gsdr::pk::mul(w[k1], w0);
                                    }
                                gsdr::pk::apply_powers<R>(w, gsdr::pk::from(tw[ROUT * n2]));
                                __builtin_amdgcn_sched_barrier(0);
                            };
                            gsdr::pk::static_for<0, T>(transform);
                        }
                    __builtin_amdgcn_sched_barrier(0);
                }
        };
        gsdr::pk::static_for<0, PAIRS>(step);
        // phase 2 writes rows over the rings: every wave's reads are done first
        __syncthreads();
    };
    auto phase1 = [&](auto qc) {
        constexpr int Q = decltype(qc)::value;
        if constexpr (split_staged<ROUT, RP>())
            {
                phase1_dma(qc);
                return;
            }
#pragma unroll
        for (int c = 0; c < CPL; ++c)
            {
                if (L % NT == 0 || wbase + c * NT < L)
                    {
                        const int n2 = min((int)threadIdx.x + c * NT, L - 1);
                        auto column_input = [&](auto n1c) {
                                constexpr int n1 = decltype(n1c)::value;
                                const int m = n1 * L + n2;
                                (void)m;
                                c2 z = gsdr::pk::conj_mul(bload(xrs, n2 * 8, n1 * L * 8), bload(crs, n2 * 8, n1 * L * 8));
#pragma unroll
                                for (int r = 1; r < ROUT; ++r)
                                    {
                                        const int so = (int)((r * M + n1 * L) * 8);
                                        const c2 y = gsdr::pk::conj_mul(bload(xrs, n2 * 8, so), bload(crs, n2 * 8, so));
                                        // W_ROUT^{r Q} = W_4^{e}, e = (r Q mod ROUT) * 4 / ROUT
                                        const int e = ((r * Q) % ROUT) * (4 / ROUT);
                                        if (e == 0)
                                            z = z + y;
                                        else if (e == 1)
                                            z = gsdr::pk::add_mi(z, y);  // z + (-i) y
                                        else if (e == 2)
                                            z = z - y;
                                        else
                                            z = gsdr::pk::sub_mi(z, y);  // z + i y
                                    }
                                if constexpr (Q > 0) z = gsdr::pk::mul_root<Q * n1, ROUT * R>(z);
                                v[0][c][n1] = z;
                        };
                        gsdr::pk::static_for<0, R>(column_input);
                        gsdr::pk::Dft<R>::run(v[0][c]);
                        // W_M^{n2 k1} = W_N^{ROUT n2 k1}; the input factor W_N^{m Q} =
                        // W_{ROUT R}^{Q n1} W_N^{Q n2} -- the first a compile-time root
                        // above, the second common to the column, so applied to its
                        // outputs here: one table read instead of R
                        if constexpr (Q > 0)
                            {
                                const c2 w0 = gsdr::pk::from(tw[Q * n2]);
#pragma unroll
                                for (int k1 = 0; k1 < R; ++k1) v[0][c][k1] = gsdr::pk::mul(v[0][c][k1], w0);
                            }
                        gsdr::pk::apply_powers<R>(v[0][c], gsdr::pk::from(tw[ROUT * n2]));
                    }
            }
    };
    auto run_phase1 = [&](auto qc) { phase1(qc); };
    if constexpr (RQ == 1)
        run_phase1(std::integral_constant<int, 0>{});
    else if constexpr (RQ == 2)
        {
            if (q == 0)
                run_phase1(std::integral_constant<int, 0>{});
            else
                run_phase1(std::integral_constant<int, 1>{});
        }
    else
        {
            switch (q)
                {
                case 0: run_phase1(std::integral_constant<int, 0>{}); break;
                case 1: run_phase1(std::integral_constant<int, 1>{}); break;
                case 2: run_phase1(std::integral_constant<int, 2>{}); break;
                default: run_phase1(std::integral_constant<int, 3>{}); break;
                }
        }
    struct Out
    {
        const float2* tw;
        float m;
        unsigned long long key;
        float* row;  // ARG with the peak ratio: the row's |R|^2 (effective window)
        uint32_t q;
        float m1;  // PPW 2: the second PRN's row maximum
        // W_L^m = W_N^{m R ROUT}
        __device__ __forceinline__ float2 twiddle(int m_) const { return tw[m_ * R * ROUT]; }
        // g: the row (k1 of transform g / R, g mod R: sub-transform q + (g / R) RQ, or PRN
        // p + g / R with PPW)
        __device__ __forceinline__ void value(c2 x, int k2, int g)
        {
            const float a = __builtin_fmaf(x.x, x.x, x.y * x.y);
            if (HALF && k2 < L / 2) return;
            if constexpr (!RP::WL && (T * R) % RP::H != 0)
                {
                    if (g >= T * R) return;  // a stale row of a partial last round
                }
            if constexpr (ARG)
                {
                    const uint32_t k1 = (uint32_t)g % (uint32_t)R, qo = q + ((uint32_t)g / (uint32_t)R) * (uint32_t)RQ;
                    // output k = qo + ROUT (k1 + R k2); effective index j = k - (N - eff)
                    const uint32_t j = qo + (uint32_t)ROUT * (k1 + (uint32_t)R * (uint32_t)k2) - (HALF ? N / 2 : 0u);
                    const unsigned long long kk = ((unsigned long long)__float_as_uint(a) << 32) | (0xffffffffu - j);
                    key = kk > key ? kk : key;
                    if (row) row[j] = a;
                }
            else if constexpr (PPW > 1)
                {
                    if (g < R)
                        m = __builtin_fmaxf(m, a);
                    else
                        m1 = __builtin_fmaxf(m1, a);
                }
            else
                m = __builtin_fmaxf(m, a);
        }
    } out{tw, 0.0f, 0ull, nullptr, q, 0.0f};
    if constexpr (ARG)
        {
            if (rowbuf) out.row = rowbuf + (size_t)(id / RQ) * (HALF ? N / 2 : N);
        }
    if constexpr (T == 1 && (RP::WL || RP::R % RP::H == 0))
        RP::template phase2<CPL>(lds, v[0], out);
    else
        RP::template phase2_multi<T, CPL>(lds, v, out);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if constexpr (ARG)
        {
            unsigned long long k = out.key;
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
                {
                    const unsigned long long t = __shfl_xor(k, o);
                    k = t > k ? t : k;
                }
            unsigned long long* sk = reinterpret_cast<unsigned long long*>(lds_raw);
            __syncthreads();  // every wave's phase-2 LDS reads are done: reuse the row buffer
            if (lane == 0) sk[wave] = k;
            __syncthreads();
            if (threadIdx.x == 0)
                {
#pragma unroll
                    for (int w2 = 1; w2 < NW; ++w2) k = sk[w2] > k ? sk[w2] : k;
                    __hip_atomic_fetch_max(&keys[id / RQ], k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            if (psum)
                {
                    // CFAR: this sub-transform's share of the Parseval sum of the row
                    // opposite the peak (pcps_acquisition.cc:531-533): sum |conj(X_opp) C|^2
                    // over inputs [q M, (q + 1) M), lane-strided, then wave and workgroup
                    // sums in a fixed order; the finish kernel adds the ROUT shares in q order
                    const uint32_t bp = id / RQ;
                    const uint32_t opp = (d + D / 2) % D;
                    float* sf = reinterpret_cast<float*>(sk + NW);
#pragma unroll
                    for (int jq = 0; jq < QPW; ++jq)
                        {
                            const uint32_t qo = q + (uint32_t)jq * RQ;
                            const c2* xo = reinterpret_cast<const c2*>(X) + xm.off(b, opp) + (size_t)qo * M;
                            const c2* co = reinterpret_cast<const c2*>(code_fft) + (size_t)p * N + (size_t)qo * M;
                            float acc = 0.0f;
                            for (uint32_t i = threadIdx.x; i < M; i += NT)
                                {
                                    const c2 y = gsdr::pk::conj_mul(xo[i], co[i]);
                                    acc = __builtin_fmaf(y.x, y.x, __builtin_fmaf(y.y, y.y, acc));
                                }
#pragma unroll
                            for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
                            if (jq > 0) __syncthreads();  // thread 0 read the previous share's slots
                            if (lane == 0) sf[wave] = acc;
                            __syncthreads();
                            if (threadIdx.x == 0)
                                {
                                    float tot = 0.0f;
#pragma unroll
                                    for (int w2 = 0; w2 < NW; ++w2) tot += sf[w2];
                                    psum[(size_t)bp * ROUT + qo] = tot;
                                }
                        }
                }
            return;
        }
    float rmax = gsdr::wave_max(out.m);
    if (lane == 0) red[wave] = rmax;
    if constexpr (PPW > 1)
        {
            const float rmax1 = gsdr::wave_max(out.m1);
            if (lane == 0) red[NW + wave] = rmax1;
        }
    __syncthreads();
    if constexpr (PPW > 1)
        {
            if (threadIdx.x == 0)
                {
                    float best1 = red[NW];
#pragma unroll
                    for (int w2 = 1; w2 < NW; ++w2) best1 = __builtin_fmaxf(best1, red[NW + w2]);
                    stats[((size_t)b * P + p + 1) * D + d] = RowStat{best1, 0u, 0.0f, 0};
                }
        }
    if (threadIdx.x == 0)
        {
            float best = red[0];
#pragma unroll
            for (int w2 = 1; w2 < NW; ++w2) best = __builtin_fmaxf(best, red[w2]);
            RowStat* st = stats + ((size_t)b * P + p) * D + d;
            if constexpr (ROUT == 1)
                *st = RowStat{best, 0u, 0.0f, 0};
            else  // non-negative floats order as their bit patterns (row zeroed by the host)
                __hip_atomic_fetch_max(reinterpret_cast<uint32_t*>(&st->max), __float_as_uint(best), __ATOMIC_RELAXED,
                    __HIP_MEMORY_SCOPE_AGENT);
        }
}

// The selected rows' results from acq_correlate_split_kernel<ARG>'s keys: code
// phase, Acq_delay_samples = fmod(indext, samples_per_code) (pcps_acquisition.cc:709)
// and the peak from the key; CFAR: the input power of the row opposite the peak by
// Parseval (:531-533, as acq_argmax_four_kernel over the whole row, same summation
// order); peak ratio: the second peak outside the +-1 chip window around the first
// (:580-604, wrapped at d_fft_size as the reference does) from the rowbuf row.
// One 256-lane workgroup per (b, p).  Not for CFAR with bit transition (the
// opposite row's half window needs its transform: acq_argmax_four_kernel).
template <int NT>
__global__ void __launch_bounds__(NT) acq_argmax_split_finish_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, gsdr_acq_result* __restrict__ res, const unsigned long long* __restrict__ keys,
    const float* __restrict__ rowbuf, const float* __restrict__ psum, uint32_t nps, AcqParams ap)
{
    constexpr int NW = NT / 64;
    __shared__ unsigned long long s_key[NW];
    __shared__ float s_sum[NW];
    const uint32_t bp = blockIdx.x;
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const uint32_t N = ap.N;
    const uint32_t d = res[bp].doppler_index;
    if (d >= ap.D) return;  // uniform
    const unsigned long long key = keys[bp];
    const uint32_t idx = 0xffffffffu - (uint32_t)(key & 0xffffffffu);
    const float peak = __uint_as_float((uint32_t)(key >> 32));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    float ip = 0.0f, second = 0.0f;
    if (ap.cfar && !ap.step_two && psum)
        {
            // the split pass's per-sub-transform shares, in sub-transform order
            float tot = 0.0f;
            for (uint32_t i = 0; i < nps; ++i) tot += psum[(size_t)bp * nps + i];
            ip = (float)((double)tot / 2.0 / (double)ap.counter);
        }
    else if (ap.cfar && !ap.step_two)
        {
            const uint32_t opp = (d + ap.D / 2) % ap.D;
            const float2* xo = X + ap.xm.off(b, opp);
            const float2* c = code_fft + (size_t)p * N;
            float acc = 0.0f;
            for (uint32_t i = threadIdx.x; i < N; i += NT)
                {
                    const float2 a = xo[i], k = c[i];
                    const float yr = a.x * k.x + a.y * k.y, yi = a.x * k.y - a.y * k.x;
                    acc = __builtin_fmaf(yr, yr, __builtin_fmaf(yi, yi, acc));
                }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
            if (lane == 0) s_sum[wave] = acc;
            __syncthreads();
            float tot = 0.0f;
#pragma unroll
            for (int w = 0; w < NW; ++w) tot += s_sum[w];
            ip = (float)((double)tot / 2.0 / (double)ap.counter);
        }
    else if (!ap.cfar)
        {
            const uint32_t eff = ap.eff;
            const float* row = rowbuf + (size_t)bp * eff;
            const int32_t ti = (int32_t)idx;
            int32_t e1 = ti - (int32_t)ap.samples_per_chip;
            int32_t e2 = ti + (int32_t)ap.samples_per_chip;
            if (e1 < 0)
                e1 = (int32_t)N + e1;
            else if (e2 >= (int32_t)N)
                e2 = e2 - (int32_t)N;
            float best = 0.0f;
            uint32_t bidx = 0;
            for (uint32_t j = threadIdx.x; j < eff; j += NT)
                {
                    const int32_t jj = (int32_t)j;
                    const bool excluded = (e1 < e2) ? (jj >= e1 && jj < e2) : (jj >= e1 || jj < e2);
                    const float m = excluded ? 0.0f : row[j];
                    if (stat_better(m, j, best, bidx))
                        {
                            best = m;
                            bidx = j;
                        }
                }
            unsigned long long k2 = ((unsigned long long)__float_as_uint(best) << 32) | (0xffffffffu - bidx);
#pragma unroll
            for (int o = 32; o > 0; o >>= 1)
                {
                    const unsigned long long t = __shfl_xor(k2, o);
                    k2 = t > k2 ? t : k2;
                }
            if (lane == 0) s_key[wave] = k2;
            __syncthreads();
#pragma unroll
            for (int w = 0; w < NW; ++w) k2 = s_key[w] > k2 ? s_key[w] : k2;
            second = __uint_as_float((uint32_t)(k2 >> 32));
        }
    if (threadIdx.x == 0)
        {
            gsdr_acq_result r = res[bp];
            r.code_phase = idx;
            r.acq_delay_samples = (double)fmodf((float)idx, ap.samples_per_code);
            r.peak = peak;
            if (ap.cfar)
                {
                    if (!ap.step_two) r.input_power = ip;
                    r.test_statistic = r.peak / r.input_power;
                }
            else
                {
                    r.second_peak = second;
                    r.test_statistic = r.peak / r.second_peak;
                }
            r.positive = r.test_statistic > ap.threshold ? 1 : 0;
            res[bp] = r;
        }
}

// After acq_reduce_kernel chose the Doppler row d* of (b, p) from the split
// kernel's row maxima: recompute row d* on the plan PT (FourStepPkPlan) -- its
// first maximum over the effective window [N - eff, N) with the reference's
// index_max rule (KERN/32f_index_max_32u.h:446-467), code_phase and
// Acq_delay_samples (pcps_acquisition.cc:709), the peak as recomputed -- and the
// CFAR power of the row opposite the peak (:531-533): by Parseval over the whole
// row, or, for the half window of bit transition, by recomputing that row too.
template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_argmax_four_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, gsdr_acq_result* __restrict__ res, const float2* __restrict__ tw,
    typename PT::PlanT plan, AcqParams ap)
{
    constexpr int NT = PT::NT;
    constexpr int NW = NT / 64;
    extern __shared__ float2 lds[];
    __shared__ unsigned long long s_key[NW];
    __shared__ float s_sum[NW];
    const uint32_t bp = blockIdx.x;
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const uint32_t N = ap.N;
    const uint32_t d = res[bp].doppler_index;
    if (d >= ap.D) return;  // uniform: no maximum found (an all-NaN grid)
    const float2* c = code_fft + (size_t)p * N;
    const int off = (int)ap.out_off;
    auto row_load = [&](const float2* x) {
        return [x, c](int i) -> float2 {
            const float2 a = x[i], k = c[i];
            return make_float2(a.x * k.x + a.y * k.y, a.x * k.y - a.y * k.x);
        };
    };
    unsigned long long key = 0ull;
    auto store = [&](int i, float2 v) {
        const int j = i - off;
        if (j < 0) return;
        const float m = __builtin_fmaf(v.x, v.x, v.y * v.y);
        const unsigned long long k = ((unsigned long long)__float_as_uint(m) << 32) | (0xffffffffu - (uint32_t)j);
        key = k > key ? k : key;
    };
    PT::run(plan, lds, tw, row_load(X + ap.xm.off(b, d)), store);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        {
            const unsigned long long t = __shfl_xor(key, o);
            key = t > key ? t : key;
        }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) s_key[wave] = key;
    __syncthreads();
#pragma unroll
    for (int w = 0; w < NW; ++w) key = s_key[w] > key ? s_key[w] : key;
    const uint32_t idx = 0xffffffffu - (uint32_t)(key & 0xffffffffu);
    const float peak = __uint_as_float((uint32_t)(key >> 32));
    float ip = 0.0f;
    if (ap.cfar && !ap.step_two)
        {
            const uint32_t opp = (d + ap.D / 2) % ap.D;
            const float2* xo = X + ap.xm.off(b, opp);
            float acc = 0.0f;
            if (off == 0)
                {
                    // accumulate(|R|^2) / fft_size = sum_k |Y_opp[k]|^2 (unnormalised R = FFT(conj Y))
                    for (uint32_t i = threadIdx.x; i < N; i += NT)
                        {
                            const float2 a = xo[i], k = c[i];
                            const float yr = a.x * k.x + a.y * k.y, yi = a.x * k.y - a.y * k.x;
                            acc = __builtin_fmaf(yr, yr, __builtin_fmaf(yi, yi, acc));
                        }
                }
            else
                {
                    auto sum_store = [&](int i, float2 v) {
                        if (i >= off) acc += __builtin_fmaf(v.x, v.x, v.y * v.y);
                    };
                    __syncthreads();  // LDS reuse by the second transform
                    PT::run(plan, lds, tw, row_load(xo), sum_store);
                }
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
            if (lane == 0) s_sum[wave] = acc;
            __syncthreads();
            float tot = 0.0f;
#pragma unroll
            for (int w = 0; w < NW; ++w) tot += s_sum[w];
            // float(accumulate) / eff, then / 2.0 / counter in double (pcps_acquisition.cc:533)
            ip = off == 0 ? (float)((double)tot / 2.0 / (double)ap.counter)
                          : (float)((double)(tot / (float)(int32_t)ap.eff) / 2.0 / (double)ap.counter);
        }
    if (threadIdx.x == 0)
        {
            gsdr_acq_result r = res[bp];
            r.code_phase = idx;
            r.acq_delay_samples = (double)fmodf((float)idx, ap.samples_per_code);
            r.peak = peak;
            if (ap.cfar)
                {
                    if (!ap.step_two) r.input_power = ip;
                    r.test_statistic = r.peak / r.input_power;
                    r.positive = r.test_statistic > ap.threshold ? 1 : 0;
                }
            res[bp] = r;
        }
}

// ---------------------------------------------------------------- K_argmax (packed f32)
// After acq_reduce_kernel chose the grid maximum's Doppler row d* of (b, p) from
// STAT-1 row maxima: recompute that row with the same packed plan and load
// functor (bit-identical values) and find its first maximum with a 64-bit key
// (|R|^2 bits, ~index) -- volk_gnsssdr_32f_index_max_32u's strict '>' scan
// (KERN/32f_index_max_32u.h:446-467) -- then write code_phase and
// Acq_delay_samples = fmod(indext, samples_per_code) (pcps_acquisition.cc:709).
template <class MP, int STAT>
__global__ void __launch_bounds__(MP::NT) acq_argmax_pk_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, gsdr_acq_result* __restrict__ res, const float2* __restrict__ tw, uint32_t D,
    uint32_t P, float samples_per_code, AcqParams ap)
{
    using gsdr::pk::c2;
    constexpr int NT = MP::NT;
    constexpr int NW = NT / 64;
    constexpr uint32_t N = MP::N;
    extern __shared__ float2 lds_raw[];
    c2* lds = reinterpret_cast<c2*>(lds_raw);
    unsigned long long* scratch = reinterpret_cast<unsigned long long*>(lds_raw + MP::lds_bytes() / sizeof(float2));
    const uint32_t bp = blockIdx.x;
    const uint32_t b = bp / P, p = bp - b * P;
    const uint32_t d = res[bp].doppler_index;
    if (d >= D) return;  // uniform: no maximum found (an all-NaN grid)
    const c2* x = reinterpret_cast<const c2*>(X) + ap.xm.off(b, d);
    const c2* c = reinterpret_cast<const c2*>(code_fft) + (size_t)p * N;
    unsigned long long key = 0ull;
    auto load = [&](int, int, int i) -> c2 { return gsdr::pk::conj_mul(x[i], c[i]); };
    auto store = [&](int i, c2 v, int) {
        const float m = __builtin_fmaf(v.x, v.x, v.y * v.y);
        const unsigned long long k = ((unsigned long long)__float_as_uint(m) << 32) | (0xffffffffu - (uint32_t)i);
        key = k > key ? k : key;
    };
    MP::template run<false>(lds, tw, load, store, [] {});
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        {
            const unsigned long long o = __shfl_xor(key, off);
            key = o > key ? o : key;
        }
    if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = key;
    __syncthreads();
    if (threadIdx.x == 0)
        {
#pragma unroll
            for (int w = 1; w < NW; ++w) key = scratch[w] > key ? scratch[w] : key;
            const uint32_t idx = 0xffffffffu - (uint32_t)(key & 0xffffffffu);
            res[bp].code_phase = idx;
            res[bp].acq_delay_samples = (double)fmodf((float)idx, samples_per_code);
        }
    if constexpr (STAT >= 2)
        {
            // CFAR input power of the row opposite the peak (pcps_acquisition.cc:531-533)
            // by Parseval: accumulate(|R|^2) / fft_size = sum_k |X_opp[k]|^2 |C[k]|^2
            if (!ap.cfar || ap.step_two) return;
            const uint32_t opp = (d + D / 2) % D;
            const c2* xo = reinterpret_cast<const c2*>(X) + ap.xm.off(b, opp);
            float acc = 0.0f;
            for (uint32_t i = threadIdx.x; i < N; i += NT)
                {
                    const c2 y = gsdr::pk::conj_mul(xo[i], c[i]);
                    acc = __builtin_fmaf(y.x, y.x, __builtin_fmaf(y.y, y.y, acc));
                }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
            float* fs = reinterpret_cast<float*>(scratch + NW);
            __syncthreads();
            if ((threadIdx.x & 63) == 0) fs[threadIdx.x >> 6] = acc;
            __syncthreads();
            if (threadIdx.x == 0)
                {
                    float tot = 0.0f;
#pragma unroll
                    for (int w = 0; w < NW; ++w) tot += fs[w];
                    // (float)((double)(acc / eff) / 2.0 / counter), acc / eff = tot
                    const float ip = (float)((double)tot / 2.0 / (double)ap.counter);
                    gsdr_acq_result r = res[bp];
                    r.input_power = ip;
                    r.test_statistic = r.peak / ip;
                    r.positive = r.test_statistic > ap.threshold ? 1 : 0;
                    res[bp] = r;
                }
        }
}

// ---------------------------------------------------------------- general path (dwells, bit transition)
// acquisition_core with max_dwells K > 1 (non-coherent accumulation of |R|^2 over
// K consecutive blocks, pcps_acquisition.cc:667-675) and/or bit_transition_flag
// (outputs [N/2, N) of each transform, :671).  One workgroup per (attempt b, d, p)
// runs the K transforms of dwells k = 0..K-1 (blocks b*K + k); each lane adds |R|^2
// into its own entries of a pooled global row (every plan maps an output index to
// the same lane in every transform, so no synchronisation is needed) and row
// statistics of the accumulated grid are emitted after every dwell:
// stats[((b*P + p)*K + k)*D + d].
__device__ __forceinline__ int pool_acquire(uint32_t* slots, int nwords)
{
    __shared__ int s_slot;
    if (threadIdx.x == 0)
        {
            int w = (int)((blockIdx.x + blockIdx.y * gridDim.x) % (unsigned)nwords);
            for (;;)
                {
                    const uint32_t cur = __hip_atomic_load(&slots[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (cur != 0xffffffffu)
                        {
                            const int bit = __builtin_ctz(~cur);
                            const uint32_t old =
                                __hip_atomic_fetch_or(&slots[w], 1u << bit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
                            if (!(old & (1u << bit)))
                                {
                                    s_slot = w * 32 + bit;
                                    break;
                                }
                        }
                    else
                        {
                            w = w + 1 == nwords ? 0 : w + 1;
                            __builtin_amdgcn_s_sleep(2);
                        }
                }
        }
    __syncthreads();
    return s_slot;
}

__device__ __forceinline__ void pool_release(uint32_t* slots, int slot)
{
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_fetch_and(&slots[slot >> 5], ~(1u << (slot & 31)), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// Cell (b, d, p) of a 1-D correlate grid over nrows = nblocks * D rows x P PRNs,
// XCD-aware for code reuse: workgroup ids go to the XCDs round-robin, so XCD x
// takes rows x, x + 8, ... and walks them PRN-group-major -- for each group of PG
// PRNs (PG | P) every one of its rows, the group's PG transforms of a row
// consecutively.  An XCD's L2 then holds PG code spectra while the X rows stream
// (at C4, N = 64000: 4 x 512 KB of codes instead of cycling through all 36) and
// each X row is fetched once per group.  Rows beyond the last multiple of 8 are
// mapped row-major.
__device__ __forceinline__ void dwell_cell(uint32_t D, uint32_t P, uint32_t nrows, uint32_t& b, uint32_t& d,
    uint32_t& p)
{
    const uint32_t id = blockIdx.x;
    const uint32_t full = nrows >> 3;
    const uint32_t PG = (P % 4u == 0u) ? 4u : ((P % 2u == 0u) ? 2u : 1u);
    uint32_t row;
    if (id < full * 8u * P)
        {
            const uint32_t xcd = id & 7u, slot = id >> 3;
            const uint32_t per_group = full * PG;
            const uint32_t pg = slot / per_group, rem = slot - pg * per_group;
            const uint32_t ri = rem / PG;
            row = ri * 8u + xcd;
            p = pg * PG + (rem - ri * PG);
        }
    else
        {
            const uint32_t t = id - full * 8u * P;
            row = full * 8u + t / P;
            p = t - (t / P) * P;
        }
    b = row / D;
    d = row - b * D;
}

template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_correlate_dwell_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, RowStat* __restrict__ stats, const float2* __restrict__ tw,
    typename PT::PlanT plan, AcqParams ap, float* __restrict__ acc_pool, uint32_t* __restrict__ acc_slots,
    int acc_words)
{
    extern __shared__ float2 lds[];
    RowStat* scratch = reinterpret_cast<RowStat*>(lds + gsdr::fft::lds_elems_dev(plan));
    const uint32_t N = plan.n;
    uint32_t b, d, p;
    dwell_cell(ap.D, ap.P, gridDim.x / ap.P, b, d, p);
    const uint32_t K = ap.dwells;
    const int slot = K > 1 ? pool_acquire(acc_slots, acc_words) : 0;
    float* acc = acc_pool + (size_t)slot * ap.eff;
    const float2* c = code_fft + (size_t)p * N;
    for (uint32_t k = 0; k < K; ++k)
        {
            const float2* x = X + ap.xm.off(b * K + k, d);
            float best = -1.0f, sum = 0.0f;
            uint32_t bidx = 0xffffffffu;
            auto load = [&](int i) -> float2 {
                float2 a = x[i], q = c[i];
                return make_float2(a.x * q.x + a.y * q.y, a.x * q.y - a.y * q.x);
            };
            auto store = [&](int i, float2 v) {
                const int j = i - (int)ap.out_off;
                if (j < 0) return;
                float m = v.x * v.x + v.y * v.y;
                if (K > 1)
                    {
                        if (k > 0) m = acc[j] + m;  // volk_32f_x2_add_32f(grid, grid, tmp)
                        acc[j] = m;
                    }
                if (stat_better(m, (uint32_t)j, best, bidx))
                    {
                        best = m;
                        bidx = (uint32_t)j;
                    }
                sum += m;
            };
            PT::run(plan, lds, tw, load, store);
            block_reduce_stat<PT::NT>(best, bidx, sum, scratch);
            if (threadIdx.x == 0) stats[(((size_t)b * ap.P + p) * K + k) * ap.D + d] = RowStat{best, bidx, sum, 0};
        }
    if (K > 1) pool_release(acc_slots, slot);
}

// One wave per (attempt b, PRN p): the statistic after every dwell k (the grid
// maximum of the accumulated grid, strict '>' scan order; CFAR input power of row
// (d*+D/2)%D divided by the dwell counter k+1, pcps_acquisition.cc:533), written to
// resk[(b*P + p)*K + k]; with CFAR also the decision (first positive dwell, else
// the last, :781-869) into res[b*P + p] with num_dwells.
__global__ void __launch_bounds__(64) acq_reduce_dwell_kernel(const RowStat* __restrict__ stats,
    gsdr_acq_result* __restrict__ resk, gsdr_acq_result* __restrict__ res, const uint32_t* __restrict__ prn_ids,
    AcqParams ap, uint64_t stamp0, uint64_t block_stride)
{
    const uint32_t bp = blockIdx.x;
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const uint32_t K = ap.dwells;
    bool done = false;
    for (uint32_t k = 0; k < K && !done; ++k)
        {
            const RowStat* s = stats + ((size_t)bp * K + k) * ap.D;
            float m = -1.0f;
            uint32_t dsel = 0xffffffffu, tsel = 0;
            for (uint32_t d = threadIdx.x; d < ap.D; d += 64)
                {
                    RowStat r = s[d];
                    if (r.max > m)
                        {
                            m = r.max;
                            dsel = d;
                            tsel = r.idx;
                        }
                }
#pragma unroll
            for (int off = 32; off > 0; off >>= 1)
                {
                    float om = __shfl_xor(m, off);
                    uint32_t od = __shfl_xor(dsel, off);
                    uint32_t ot = __shfl_xor(tsel, off);
                    if (stat_better(om, od, m, dsel))
                        {
                            m = om;
                            dsel = od;
                            tsel = ot;
                        }
                }
            gsdr_acq_result r;
            r.prn = prn_ids[p];
            r.doppler_index = dsel;
            r.code_phase = tsel;
            r.doppler_hz = doppler_of(ap, dsel);
            r.peak = m;
            r.second_peak = 0.0f;
            r.input_power = 0.0f;
            r.test_statistic = 0.0f;
            r.acq_delay_samples = (double)fmodf((float)tsel, ap.samples_per_code);
            r.samplestamp = stamp0 + (uint64_t)(b * K + k) * block_stride;
            r.positive = 0;
            r.num_dwells = (int32_t)(k + 1);
            if (ap.cfar)
                {
                    const uint32_t opp = (dsel + ap.D / 2) % ap.D;
                    const float acc = s[opp].sum;
                    const float ip = ap.step_two ? ap.ip2
                                                 : (float)((double)(acc / (float)(int32_t)ap.eff) / 2.0 / (double)(k + 1));
                    r.input_power = ip;
                    r.test_statistic = m / ip;
                    r.positive = r.test_statistic > ap.threshold ? 1 : 0;
                    done = r.positive || k + 1 == K;
                    if (done && threadIdx.x == 0) res[bp] = r;
                }
            if (threadIdx.x == 0) resk[(size_t)bp * K + k] = r;
        }
}

// Peak-ratio statistic per dwell: the accumulated row d*_k over dwells 0..k,
// maximum outside the exclusion window (as acq_second_peak_kernel).  grid (K, B*P).
template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_second_peak_dwell_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, gsdr_acq_result* __restrict__ resk, const float2* __restrict__ tw,
    typename PT::PlanT plan, AcqParams ap, float* __restrict__ acc_pool, uint32_t* __restrict__ acc_slots,
    int acc_words)
{
    extern __shared__ float2 lds[];
    RowStat* scratch = reinterpret_cast<RowStat*>(lds + gsdr::fft::lds_elems_dev(plan));
    const uint32_t kk = blockIdx.x, bp = blockIdx.y;
    const uint32_t K = ap.dwells;
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const uint32_t N = plan.n;
    gsdr_acq_result* rr = resk + (size_t)bp * K + kk;
    const uint32_t d = rr->doppler_index;
    const int32_t ti = (int32_t)rr->code_phase;
    // the reference wraps the exclusion window at d_fft_size even when the rows
    // hold the effective N/2 outputs (bit transition; :580-590)
    const int32_t E = (int32_t)ap.N;
    int32_t e1 = ti - (int32_t)ap.samples_per_chip;
    int32_t e2 = ti + (int32_t)ap.samples_per_chip;
    if (e1 < 0)
        e1 = E + e1;
    else if (e2 >= E)
        e2 = e2 - E;
    const int slot = kk > 0 ? pool_acquire(acc_slots, acc_words) : 0;
    float* acc = acc_pool + (size_t)slot * ap.eff;
    const float2* c = code_fft + (size_t)p * N;
    float best = 0.0f, sum = 0.0f;
    uint32_t bidx = 0;
    for (uint32_t k = 0; k <= kk; ++k)
        {
            const float2* x = X + ap.xm.off(b * K + k, d);
            const bool last = k == kk;
            auto load = [&](int i) -> float2 {
                float2 a = x[i], q = c[i];
                return make_float2(a.x * q.x + a.y * q.y, a.x * q.y - a.y * q.x);
            };
            auto store = [&](int i, float2 v) {
                const int j = i - (int)ap.out_off;
                if (j < 0) return;
                float m = v.x * v.x + v.y * v.y;
                if (kk > 0)
                    {
                        if (k > 0) m = acc[j] + m;
                        if (!last) acc[j] = m;
                    }
                if (last)
                    {
                        const bool excluded = (e1 < e2) ? (j >= e1 && j < e2) : (j >= e1 || j < e2);
                        if (excluded) m = 0.0f;
                        if (stat_better(m, (uint32_t)j, best, bidx))
                            {
                                best = m;
                                bidx = (uint32_t)j;
                            }
                    }
            };
            PT::run(plan, lds, tw, load, store);
        }
    block_reduce_stat<PT::NT>(best, bidx, sum, scratch);
    if (threadIdx.x == 0)
        {
            gsdr_acq_result r = *rr;
            r.second_peak = best;
            r.test_statistic = r.peak / best;
            r.positive = r.test_statistic > ap.threshold ? 1 : 0;
            *rr = r;
        }
    if (kk > 0) pool_release(acc_slots, slot);
}

// Peak-ratio decision over the dwells: the first positive dwell, else the last.
__global__ void acq_decide_kernel(const gsdr_acq_result* __restrict__ resk, gsdr_acq_result* __restrict__ res,
    uint32_t K, uint32_t n)
{
    const uint32_t bp = blockIdx.x * blockDim.x + threadIdx.x;
    if (bp >= n) return;
    uint32_t k = 0;
    while (k + 1 < K && !resk[(size_t)bp * K + k].positive) ++k;
    res[bp] = resk[(size_t)bp * K + k];
}

// ---------------------------------------------------------------- dwell per call (gsdr_acq_run_dwell)
// acquisition_core's own dwell loop: one call per general_work block, the |R|^2
// grid kept across calls (pcps_acquisition.cc:637-680: the first dwell writes
// d_magnitude_grid, later dwells add into it with volk_32f_x2_add_32f) in a
// device-resident grid[p][d][eff]; the statistic of the accumulated grid after
// every call (:689-696) with the dwell counter as the CFAR divisor (:534).
// One workgroup per (d, p) of one block.
template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_dwell_grid_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, RowStat* __restrict__ stats, const float2* __restrict__ tw,
    typename PT::PlanT plan, AcqParams ap, float* __restrict__ grid, uint32_t dwell)
{
    extern __shared__ float2 lds[];
    RowStat* scratch = reinterpret_cast<RowStat*>(lds + gsdr::fft::lds_elems_dev(plan));
    const uint32_t N = plan.n;
    const uint32_t d = blockIdx.x / ap.P, p = blockIdx.x - d * ap.P;
    float* row = grid + ((size_t)p * ap.D + d) * ap.eff;
    const float2* x = X + ap.xm.off(0, d);
    const float2* c = code_fft + (size_t)p * N;
    float best = -1.0f, sum = 0.0f;
    uint32_t bidx = 0xffffffffu;
    auto load = [&](int i) -> float2 {
        float2 a = x[i], q = c[i];
        return make_float2(a.x * q.x + a.y * q.y, a.x * q.y - a.y * q.x);
    };
    auto store = [&](int i, float2 v) {
        const int j = i - (int)ap.out_off;
        if (j < 0) return;
        float m = v.x * v.x + v.y * v.y;
        if (dwell > 0) m = row[j] + m;
        row[j] = m;
        if (stat_better(m, (uint32_t)j, best, bidx))
            {
                best = m;
                bidx = (uint32_t)j;
            }
        sum += m;
    };
    PT::run(plan, lds, tw, load, store);
    block_reduce_stat<PT::NT>(best, bidx, sum, scratch);
    if (threadIdx.x == 0) stats[(size_t)p * ap.D + d] = RowStat{best, bidx, sum, 0};
}

// first_vs_second_peak_statistic (:546-612) on the accumulated grid: row d* with
// the +-samples_per_chip window zeroed (wrap at d_fft_size, :580-590), first
// maximum of the rest.  One workgroup per PRN.
__global__ void __launch_bounds__(256) acq_grid_second_peak_kernel(const float* __restrict__ grid,
    gsdr_acq_result* __restrict__ res, AcqParams ap)
{
    __shared__ RowStat scratch[4];
    const uint32_t p = blockIdx.x;
    const uint32_t d = res[p].doppler_index;
    const int32_t ti = (int32_t)res[p].code_phase;
    const int32_t E = (int32_t)ap.N;
    int32_t e1 = ti - (int32_t)ap.samples_per_chip;
    int32_t e2 = ti + (int32_t)ap.samples_per_chip;
    if (e1 < 0)
        e1 = E + e1;
    else if (e2 >= E)
        e2 = e2 - E;
    const float* row = grid + ((size_t)p * ap.D + d) * ap.eff;
    float best = 0.0f, sum = 0.0f;
    uint32_t bidx = 0;
    for (uint32_t j = threadIdx.x; j < ap.eff; j += 256)
        {
            const int32_t jj = (int32_t)j;
            const bool excluded = (e1 < e2) ? (jj >= e1 && jj < e2) : (jj >= e1 || jj < e2);
            const float m = excluded ? 0.0f : row[j];
            if (stat_better(m, j, best, bidx))
                {
                    best = m;
                    bidx = j;
                }
        }
    block_reduce_stat<256>(best, bidx, sum, scratch);
    if (threadIdx.x == 0)
        {
            gsdr_acq_result r = res[p];
            r.second_peak = best;
            r.test_statistic = r.peak / best;
            r.positive = r.test_statistic > ap.threshold ? 1 : 0;
            res[p] = r;
        }
}

// ---------------------------------------------------------------- K_forward (packed f32)
// X_{b,d} = FFT(x_b .* w_d) on the packed plan (the N = 4000 path, with the packed
// correlate variants).  Grid (B, D) with the block index fastest, as
// acq_forward_kernel.
template <class MP, int IT>
__global__ void __launch_bounds__(MP::NT) acq_forward_pk_kernel(const void* __restrict__ iq, uint64_t block_stride,
    const float2* __restrict__ wipe, float2* __restrict__ X, const float2* __restrict__ tw, uint32_t consumed, XMap xm)
{
    using gsdr::pk::c2;
    extern __shared__ float2 lds_raw[];
    c2* lds = reinterpret_cast<c2*>(lds_raw);
    const uint32_t b = blockIdx.x, d = blockIdx.y;
    constexpr uint32_t N = MP::N;
    const size_t base = (size_t)b * block_stride;
    const c2* w = reinterpret_cast<const c2*>(wipe) + (size_t)d * N;
    c2* out = reinterpret_cast<c2*>(X) + xm.off(b, d);
    const int ext = (int)(xm.stride - N);  // bins repeated after N - 1 (XMap)
    auto load = [&](int, int, int i) -> c2 {
        if (i >= (int)consumed) return c2{0.f, 0.f};
        return gsdr::pk::mul(gsdr::pk::from(load_item<IT>(iq, base + i)), w[i]);
    };
    auto store = [&](int i, c2 v, int) {
        out[i] = v;
        if (i < ext) out[N + i] = v;
    };
    MP::run(lds, tw, load, store, [] {});
}

// ---------------------------------------------------------------- K_reduce
// One wave per (b, p).  Rows are scanned in increasing d by each lane and merged
// with the (max desc, d asc) order, reproducing the reference's strict '>' scan.
__global__ void __launch_bounds__(64) acq_reduce_kernel(const RowStat* __restrict__ stats,
    gsdr_acq_result* __restrict__ res, const uint32_t* __restrict__ prn_ids, AcqParams ap, uint64_t stamp0,
    uint64_t block_stride)
{
    const uint32_t bp = blockIdx.x;  // b*P + p
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const RowStat* s = stats + (size_t)bp * ap.D;
    float m = -1.0f;
    uint32_t dsel = 0xffffffffu, tsel = 0;
    for (uint32_t d = threadIdx.x; d < ap.D; d += 64)
        {
            RowStat r = s[d];
            if (r.max > m)
                {
                    m = r.max;
                    dsel = d;
                    tsel = r.idx;
                }
        }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1)
        {
            float om = __shfl_xor(m, off);
            uint32_t od = __shfl_xor(dsel, off);
            uint32_t ot = __shfl_xor(tsel, off);
            if (stat_better(om, od, m, dsel))
                {
                    m = om;
                    dsel = od;
                    tsel = ot;
                }
        }
    if (threadIdx.x != 0) return;
    gsdr_acq_result r;
    r.prn = prn_ids[p];
    r.doppler_index = dsel;
    r.code_phase = tsel;
    r.doppler_hz = doppler_of(ap, dsel);
    r.peak = m;
    r.second_peak = 0.0f;
    r.input_power = 0.0f;
    r.test_statistic = 0.0f;
    r.acq_delay_samples = (double)fmodf((float)tsel, ap.samples_per_code);
    r.samplestamp = stamp0 + (uint64_t)b * block_stride;
    r.positive = 0;
    r.num_dwells = (int32_t)ap.counter;
    if (ap.cfar)
        {
            const uint32_t opp = (dsel + ap.D / 2) % ap.D;
            const float acc = s[opp].sum;
            // float(accumulate) / int32 in float, then / 2.0 / counter in double (pcps_acquisition.cc:533)
            const float ip =
                ap.step_two ? ap.ip2 : (float)((double)(acc / (float)(int32_t)ap.eff) / 2.0 / (double)ap.counter);
            r.input_power = ip;
            r.test_statistic = m / ip;
            r.positive = r.test_statistic > ap.threshold ? 1 : 0;
        }
    res[bp] = r;
}

// ---------------------------------------------------------------- K_second
// Peak-ratio statistic: recompute row d* of (b, p) and take the maximum outside
// the cyclic exclusion range [e1, e2) built as in pcps_acquisition.cc:580-604.
template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_second_peak_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, gsdr_acq_result* __restrict__ res, const float2* __restrict__ tw,
    typename PT::PlanT plan, AcqParams ap)
{
    extern __shared__ float2 lds[];
    RowStat* scratch = reinterpret_cast<RowStat*>(lds + gsdr::fft::lds_elems_dev(plan));
    const uint32_t bp = blockIdx.x;
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const uint32_t N = plan.n;
    const uint32_t d = res[bp].doppler_index;
    const int32_t ti = (int32_t)res[bp].code_phase;
    // the window over the effective outputs j = i - out_off (bit transition: the
    // second half); the reference wraps it at d_fft_size all the same (:580-590)
    int32_t e1 = ti - (int32_t)ap.samples_per_chip;
    int32_t e2 = ti + (int32_t)ap.samples_per_chip;
    if (e1 < 0)
        e1 = (int32_t)N + e1;
    else if (e2 >= (int32_t)N)
        e2 = e2 - (int32_t)N;
    const float2* x = X + ap.xm.off(b, d);
    const float2* c = code_fft + (size_t)p * N;
    float best = 0.0f, sum = 0.0f;
    uint32_t bidx = 0;
    auto load = [&](int i) -> float2 {
        float2 a = x[i], k = c[i];
        return make_float2(a.x * k.x + a.y * k.y, a.x * k.y - a.y * k.x);
    };
    auto store = [&](int i, float2 v) {
        const int j = i - (int)ap.out_off;
        if (j < 0) return;
        const bool excluded = (e1 < e2) ? (j >= e1 && j < e2) : (j >= e1 || j < e2);
        const float m = excluded ? 0.0f : v.x * v.x + v.y * v.y;
        if (stat_better(m, (uint32_t)j, best, bidx))
            {
                best = m;
                bidx = (uint32_t)j;
            }
    };
    PT::run(plan, lds, tw, load, store);
    block_reduce_stat<PT::NT>(best, bidx, sum, scratch);
    if (threadIdx.x == 0)
        {
            gsdr_acq_result r = res[bp];
            r.second_peak = best;
            r.test_statistic = r.peak / best;
            r.positive = r.test_statistic > ap.threshold ? 1 : 0;
            res[bp] = r;
        }
}

// Peak ratio on the split path in one pass over the selected row: recompute row d*
// of (b, p) on PT once (acq_argmax_four_kernel + acq_second_peak_kernel recomputed
// it twice), keep its |R|^2 in the workgroup's row of rowbuf while finding the
// first maximum (index_max rule), then scan that row again for the maximum
// outside the exclusion window around it (pcps_acquisition.cc:580-604, wrapped at
// d_fft_size as the reference does).  Values bit-identical to the two kernels'.
template <class PT>
__global__ void __launch_bounds__(PT::NT) acq_argmax_second_four_kernel(const float2* __restrict__ X,
    const float2* __restrict__ code_fft, gsdr_acq_result* __restrict__ res, const float2* __restrict__ tw,
    typename PT::PlanT plan, AcqParams ap, float* __restrict__ rowbuf)
{
    constexpr int NT = PT::NT;
    constexpr int NW = NT / 64;
    extern __shared__ float2 lds[];
    __shared__ unsigned long long s_key[NW];
    const uint32_t bp = blockIdx.x;
    const uint32_t b = bp / ap.P, p = bp - b * ap.P;
    const uint32_t N = ap.N;
    const uint32_t d = res[bp].doppler_index;
    if (d >= ap.D) return;  // uniform: no maximum found (an all-NaN grid)
    const float2* x = X + ap.xm.off(b, d);
    const float2* c = code_fft + (size_t)p * N;
    const int off = (int)ap.out_off;
    const uint32_t eff = N - (uint32_t)off;
    float* row = rowbuf + (size_t)bp * N;
    auto load = [&](int i) -> float2 {
        const float2 a = x[i], k = c[i];
        return make_float2(a.x * k.x + a.y * k.y, a.x * k.y - a.y * k.x);
    };
    unsigned long long key = 0ull;
    auto store = [&](int i, float2 v) {
        const int j = i - off;
        if (j < 0) return;
        const float m = __builtin_fmaf(v.x, v.x, v.y * v.y);
        row[j] = m;
        const unsigned long long k = ((unsigned long long)__float_as_uint(m) << 32) | (0xffffffffu - (uint32_t)j);
        key = k > key ? k : key;
    };
    PT::run(plan, lds, tw, load, store);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        {
            const unsigned long long t = __shfl_xor(key, o);
            key = t > key ? t : key;
        }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) s_key[wave] = key;
    __syncthreads();  // also orders every lane's row stores before the scan below
#pragma unroll
    for (int w = 0; w < NW; ++w) key = s_key[w] > key ? s_key[w] : key;
    const uint32_t idx = 0xffffffffu - (uint32_t)(key & 0xffffffffu);
    const float peak = __uint_as_float((uint32_t)(key >> 32));
    // second peak (acq_second_peak_kernel's window and tie rule)
    const int32_t ti = (int32_t)idx;
    int32_t e1 = ti - (int32_t)ap.samples_per_chip;
    int32_t e2 = ti + (int32_t)ap.samples_per_chip;
    if (e1 < 0)
        e1 = (int32_t)N + e1;
    else if (e2 >= (int32_t)N)
        e2 = e2 - (int32_t)N;
    float best = 0.0f;
    uint32_t bidx = 0;
    for (uint32_t j = threadIdx.x; j < eff; j += NT)
        {
            const int32_t jj = (int32_t)j;
            const bool excluded = (e1 < e2) ? (jj >= e1 && jj < e2) : (jj >= e1 || jj < e2);
            const float m = excluded ? 0.0f : row[j];
            if (stat_better(m, j, best, bidx))
                {
                    best = m;
                    bidx = j;
                }
        }
    __syncthreads();  // s_key reuse
    unsigned long long k2 = ((unsigned long long)__float_as_uint(best) << 32) | (0xffffffffu - bidx);
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        {
            const unsigned long long t = __shfl_xor(k2, o);
            k2 = t > k2 ? t : k2;
        }
    if (lane == 0) s_key[wave] = k2;
    __syncthreads();
    if (threadIdx.x == 0)
        {
#pragma unroll
            for (int w = 0; w < NW; ++w) k2 = s_key[w] > k2 ? s_key[w] : k2;
            gsdr_acq_result r = res[bp];
            r.code_phase = idx;
            r.acq_delay_samples = (double)fmodf((float)idx, ap.samples_per_code);
            r.peak = peak;
            r.second_peak = __uint_as_float((uint32_t)(k2 >> 32));
            r.test_statistic = r.peak / r.second_peak;
            r.positive = r.test_statistic > ap.threshold ? 1 : 0;
            res[bp] = r;
        }
}

}  // namespace

// ====================================================================== handle
struct gsdr_acq
{
    int device{0};
    gsdr_acq_conf conf{};
    uint32_t N{0}, D{0}, consumed{0}, lead{0};
    uint32_t K{1};       // max_dwells
    int wipe_mode{GSDR_WIPE_EXACT};  // carrier model of the Doppler grid (gsdr_acq_set_wipeoff)
    XMap xm_grid{};      // forward-spectrum layout of the main Doppler grid (rebuild_wipeoffs)
    XMap xm{};           // the layout of the launches being issued (set by dispatch)
    uint32_t eff{0};     // effective FFT size (outputs [N - eff, N))
    bool general{false}; // dwells > 1 or bit transition: the general kernels
    gsdr_acq_result* d_resk{nullptr};  // per-dwell results (general path)
    float* d_acc{nullptr};             // pooled |R|^2 accumulation rows (general path)
    uint32_t* d_acc_slots{nullptr};
    int acc_words{0};
    float threshold{0.0f};
    int nt{256};
    int variant{0};
    int corr_variant{0};      // 0: the generic LDS kernels; >0: a GSDR_PK_VARIANTS id (packed forward + correlate)
    int split{0};             // >0: the single-dwell split register four-step correlate (acq_split.hip)
    uint32_t split_pgs{1};    // its PRN group per XCD pass
    int corr_stat{0};         // the variant's row statistic (1/2: argmax recomputed by acq_argmax_pk_kernel)
    size_t corr_lds_bytes{0};
    Plan plan{};
    gsdr::fft::Plan4 plan4{};  // four-step plan (variants 20-22, N beyond one workgroup's LDS)
    size_t lds_bytes{0};
    hipStream_t stream{nullptr};
    float2* d_tw{nullptr};
    float2* d_wipe{nullptr};
    float2* d_wipe_grid{nullptr};  // the main grid's wipe-off rows (d_wipe points elsewhere during step two)
    float2* d_code_fft{nullptr};
    float2* d_code_stage{nullptr};
    uint32_t* d_prn{nullptr};
    uint32_t nprn{0};
    float2* d_X{nullptr};
    RowStat* d_stats{nullptr};
    gsdr_acq_result* d_res{nullptr};
    // gsdr_acq_submit_stream / gsdr_acq_collect: up to kSubs submissions in flight,
    // each with its pinned results (max_blocks x max_prns), completion event and shape;
    // a later submission's grid reuses d_res on the same stream, ordered after the
    // earlier one's copy out of it
    static constexpr int kSubs = 2;
    gsdr_acq_result* h_res[kSubs]{};
    hipEvent_t sub_done[kSubs]{};
    uint32_t sub_blocks[kSubs]{}, sub_nprn[kSubs]{};
    int sub_head{0}, sub_count{0};
    void* d_iq{nullptr};
    float* d_grid{nullptr};
    float* d_rowbuf{nullptr};  // split path, peak ratio: the selected rows' |R|^2 (max_blocks x max_prns x N)
    unsigned long long* d_keys{nullptr};  // split path: the selected rows' first-maximum keys (max_blocks x max_prns)
    float* d_psum{nullptr};               // split path, CFAR: Parseval shares per sub-transform (max_blocks x max_prns x 4)
    float2* d_fscratch{nullptr};  // split path: the two-launch forward's column-DFT rows (max_blocks x D x N)
    float* d_dgrid{nullptr};     // gsdr_acq_run_dwell: the |R|^2 grid kept across calls (max_prns x D x eff)
    float2* d_tw_sub{nullptr};   // four-step: W_N2 table
    float2* d_scratch{nullptr};  // four-step: slot rows of N complex
    uint32_t* d_slots{nullptr};  // four-step: slot occupancy bitmap
    // stage profiling (gsdr_acq_set_profiling)
    struct ProfRec
    {
        hipEvent_t a, b;
        int stage;
    };
    bool profiling{false};
    std::vector<ProfRec> prof_recs;
    std::vector<hipEvent_t> prof_pool;
    // make_two_steps (gsdr_acq_set_step_two / gsdr_acq_run_step_two)
    struct StepTwo
    {
        uint32_t nbins{0};       // num_doppler_bins_step2
        float step{0.0f};        // doppler_step2
        float pfa2{0.0f};
        float threshold{0.0f};   // calculate_threshold with d_step_two
        float2* d_wipe{nullptr}; // max_prns x nbins rows of N
        float* d_freq{nullptr};
        bool active{false};      // set while the per-PRN step-two launches are issued
        float center{0.0f}, ip{0.0f};
    } st2;
    std::mutex mu;
};

namespace
{

using gsdr::fft::FourStepPlan;
using gsdr::fft::RuntimePlan;
using gsdr::fft::StaticPlan;

size_t item_bytes(int it) { return it == GSDR_ITEM_CSHORT ? 4 : (it == GSDR_ITEM_IBYTE ? 2 : 8); }

// FFT variants (gsdr_acq::variant): 1-4 compile-time plans for the sample rates
// GNSS front-ends use (2/4/8/16 Msps at 1 ms, acq_v_static.hip), 10-12 runtime
// LDS plans for every other 2^a3^b5^c size (acq_v_runtime.hip), 20/22 the
// four-step FFT beyond one workgroup's LDS (acq_v_four.hip).


// Packed-f32 correlate (and forward / argmax) variants, one per compile-time FFT
// size (default_pk_variant; GSDR_ACQ_CORR_VARIANT selects one for tests):
// (id, plan, PRNs per workgroup, waves-per-EU hint, row statistic: 1 max + sum
// with the argmax recomputed for the selected row, 2 max only with the CFAR row
// sum by Parseval -- see acq_correlate_pk_kernel).  93 runs the correlate on the
// register four-step (acq_correlate_reg_kernel, N = 16000, PRN-group-major XCD
// walk) and its forward / argmax passes on the listed plan; 94 the same with
// wave-local row transforms (RegFourStep H = 0).  The alternatives measured in
// rounds 1-4 and removed: other radix orders, per-stage twiddle
// tables (-23 %) and LDS root copies (-2.5 %), padded layouts, late or dropped
// barriers, 5 waves per SIMD (with spills -19 %; without, the first-stage products
// in two halves, -2 %), 3 / 2 workgroups per CU (-8 % / -26 %), per-wave atomic row
// maxima (-2 %), multi-transform workgroups: variant 70 at 104 VGPRs runs 4
// workgroups (16 waves) per CU, where the CU's issue, not latency, bounds it.
#define GSDR_PK_VARIANTS(X)                                              \
    X(61, (gsdr::pk::PkPlan<512, true, 20, 20, 20>), 1, 1, 1)           \
    X(62, (gsdr::pk::PkPlan<256, true, 20, 10, 10>), 1, 1, 1)           \
    X(93, (gsdr::pk::PkPlan<1024, 1, 16, 10, 10, 10>), 1, 1, 2)         \
    X(94, (gsdr::pk::PkPlan<1024, 1, 16, 10, 10, 10>), 1, 1, 2)         \
    X(70, (gsdr::pk::PkPlan<256, 1, 25, 16, 10>), 1, 1, 2)

template <class PT>
int set_lds_attrs(size_t bytes)
{
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_code_fft_kernel<PT>, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward_kernel<PT, GSDR_ITEM_GR_COMPLEX>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward_kernel<PT, GSDR_ITEM_CSHORT>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward_kernel<PT, GSDR_ITEM_IBYTE>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_kernel<PT, false>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_kernel<PT, true>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_second_peak_kernel<PT>, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_correlate_dwell_kernel<PT>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_second_peak_dwell_kernel<PT>,
        hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
    GSDR_HIP(hipFuncSetAttribute((const void*)acq_dwell_grid_kernel<PT>, hipFuncAttributeMaxDynamicSharedMemorySize,
        (int)bytes));
    if constexpr (std::is_same<typename PT::PlanT, gsdr::fft::Plan4>::value)
        {
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_argmax_four_kernel<PT>,
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
            GSDR_HIP(hipFuncSetAttribute((const void*)acq_argmax_second_four_kernel<PT>,
                hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes));
            if constexpr (requires_subplan<PT>::value)
                GSDR_HIP(hipFuncSetAttribute((const void*)acq_forward4_rows_kernel<PT>,
                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)PT::SubPlan::lds_bytes()));
        }
    return GSDR_OK;
}

AcqParams params_of(const gsdr_acq* a)
{
    AcqParams ap{};
    ap.xm = a->xm;
    ap.N = a->N;
    ap.consumed = a->consumed;
    ap.lead_zeros = a->lead;
    ap.D = a->D;
    ap.P = a->nprn;
    ap.doppler_max = a->conf.doppler_max;
    ap.doppler_center = a->conf.doppler_center;
    ap.doppler_step = (int32_t)a->conf.doppler_step;
    ap.samples_per_code = a->conf.samples_per_code;
    ap.samples_per_chip = a->conf.samples_per_chip;
    ap.dwells = a->K;
    ap.threshold = a->threshold;
    ap.cfar = a->conf.pfa > 0.0f ? 1 : 0;
    ap.eff = a->eff;
    ap.out_off = a->N - a->eff;
    ap.counter = a->K;
    if (a->st2.active)
        {
            ap.step_two = 1;
            ap.center2 = a->st2.center;
            ap.step2 = a->st2.step;
            ap.half2 = (float)std::floor((double)a->st2.nbins / 2.0);
            ap.ip2 = a->st2.ip;
            ap.threshold = a->st2.threshold;
        }
    return ap;
}

// The forward-spectrum reuse of the main grid (XMap): with the exact carrier and
// doppler_step * N / fs = p / q in lowest terms, q <= D / 2, the q spectra of
// Doppler bins 0..q-1 (each extended by E = ((D - 1) / q) p bins) hold every row;
// else the plain layout.  GSDR_ACQ_XSHIFT=0 keeps the plain layout.
XMap grid_xmap(const gsdr_acq* a)
{
    XMap plain{a->D, 0u, a->N};
    if (a->wipe_mode != GSDR_WIPE_EXACT) return plain;
    if (const char* e = std::getenv("GSDR_ACQ_XSHIFT"))
        if (std::atoi(e) == 0) return plain;
    const int64_t fs = a->conf.fs_in;
    if (fs <= 0) return plain;
    int64_t num = (int64_t)a->conf.doppler_step * (int64_t)a->N, den = fs;
    int64_t g0 = num, g1 = den;
    while (g1)  // gcd
        {
            const int64_t t = g0 % g1;
            g0 = g1;
            g1 = t;
        }
    if (g0 <= 0) return plain;
    const int64_t p = num / g0, q = den / g0;
    if (q < 1 || 2 * q > (int64_t)a->D) return plain;
    const int64_t ext = ((int64_t)(a->D - 1) / q) * p;
    // the forward stores mirror bins i < N after bin N - 1 (out[N + i], i < ext), so
    // a Doppler span wider than fs (ext > N) would leave rows reading unwritten bins
    if (ext > (int64_t)a->N) return plain;
    // the stored spectra must fit the plain layout's allocation
    if (q * ((int64_t)a->N + ext) > (int64_t)a->D * (int64_t)a->N) return plain;
    return XMap{(uint32_t)q, (uint32_t)p, (uint32_t)(a->N + ext)};
}

int rebuild_wipeoffs(gsdr_acq* a)
{
    a->xm_grid = grid_xmap(a);
    // rows 0..q-1 suffice with the reuse (the other rows would be their shifts)
    hipLaunchKernelGGL(acq_wipeoff_kernel, dim3(a->xm_grid.q), dim3(256), 0, a->stream, a->d_wipe, a->N,
        (float)a->conf.fs_in, a->conf.doppler_max, a->conf.doppler_center, (int32_t)a->conf.doppler_step,
        a->conf.doppler_bias, (const float*)nullptr, a->wipe_mode);
    GSDR_HIP(hipGetLastError());
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

void compute_threshold(gsdr_acq* a)
{
    // calculate_threshold, pcps_acquisition.cc:894-909: effective FFT size (N/2
    // with bit transition) x bins, 2*dwells degrees of freedom (max_dwells is 1
    // with bit transition)
    const float pfa = a->conf.pfa;
    if (pfa <= 0.0f) return;
    const int num_bins = (int)(a->eff * a->D);
    const double p = std::pow(1.0 - (double)pfa, 1.0 / (double)(float)num_bins);
    a->threshold = (float)(2.0 * gsdr::gamma_p_inv_int(2 * (int)a->conf.max_dwells, p));
}

// calculate_threshold with d_step_two (:894-909): pfa2 and the narrow bin count;
// with pfa2 <= 0 the reference returns early and keeps the first-step threshold.
float step_two_threshold(const gsdr_acq* a)
{
    const float pfa = a->st2.pfa2;
    if (pfa <= 0.0f) return a->threshold;
    const int num_bins = (int)(a->eff * a->st2.nbins);
    const double p = std::pow(1.0 - (double)pfa, 1.0 / (double)(float)num_bins);
    return (float)(2.0 * gsdr::gamma_p_inv_int(2 * (int)a->conf.max_dwells, p));
}

// Event bracket around one stage launch when profiling is on.
struct StageTimer
{
    gsdr_acq* a;
    hipStream_t s;
    hipEvent_t ev0{nullptr};
    StageTimer(gsdr_acq* a_, hipStream_t s_) : a(a_), s(s_) {}
    hipEvent_t take()
    {
        hipEvent_t e = nullptr;
        if (!a->prof_pool.empty())
            {
                e = a->prof_pool.back();
                a->prof_pool.pop_back();
            }
        else if (hipEventCreate(&e) != hipSuccess)
            e = nullptr;
        return e;
    }
    void begin()
    {
        if (!a->profiling) return;
        ev0 = take();
        if (ev0) (void)hipEventRecord(ev0, s);
    }
    void end(int stage)
    {
        if (!a->profiling || !ev0) return;
        hipEvent_t ev1 = take();
        if (!ev1) return;
        (void)hipEventRecord(ev1, s);
        a->prof_recs.push_back({ev0, ev1, stage});
        ev0 = nullptr;
    }
};

}  // namespace

// Defined in the variant translation units (one per plan-type group, compiled in
// parallel): acq_pk.hip, acq_v_static.hip, acq_v_runtime.hip, acq_v_four.hip.
namespace gsdr_acq_impl
{
int launch_corr_variant(gsdr_acq* a, uint32_t nblocks, hipStream_t s);
int launch_argmax_variant(gsdr_acq* a, uint32_t nblocks, gsdr_acq_result* res, hipStream_t s);
int launch_forward_pk(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, hipStream_t s);
int setup_corr_variant(gsdr_acq* a, int v);
int setup_split(gsdr_acq* a);
int launch_split(gsdr_acq* a, uint32_t nblocks, hipStream_t s);
int launch_split_argmax(gsdr_acq* a, uint32_t nblocks, gsdr_acq_result* res, hipStream_t s);
int dispatch_static(gsdr_acq* a, int op, const void* iq, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, uint32_t aux);
int dispatch_runtime(gsdr_acq* a, int op, const void* iq, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, uint32_t aux);
int dispatch_four(gsdr_acq* a, int op, const void* iq, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, uint32_t aux);
}  // namespace gsdr_acq_impl

namespace
{
using gsdr_acq_impl::launch_corr_variant;
using gsdr_acq_impl::launch_forward_pk;

template <class PT>
const typename PT::PlanT& plan_of(const gsdr_acq* a)
{
    if constexpr (std::is_same<typename PT::PlanT, gsdr::fft::Plan4>::value)
        return a->plan4;
    else
        return a->plan;
}

template <class PT>
void launch_forward(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, hipStream_t s)
{
    if (item_type == GSDR_ITEM_GR_COMPLEX)
        hipLaunchKernelGGL((acq_forward_kernel<PT, GSDR_ITEM_GR_COMPLEX>), dim3(nblocks, a->xm.q), dim3(PT::NT),
            a->lds_bytes, s, iq, stride, a->d_wipe, a->d_X, a->d_tw, plan_of<PT>(a), a->consumed, a->xm);
    else if (item_type == GSDR_ITEM_CSHORT)
        hipLaunchKernelGGL((acq_forward_kernel<PT, GSDR_ITEM_CSHORT>), dim3(nblocks, a->xm.q), dim3(PT::NT),
            a->lds_bytes, s, iq, stride, a->d_wipe, a->d_X, a->d_tw, plan_of<PT>(a), a->consumed, a->xm);
    else
        hipLaunchKernelGGL((acq_forward_kernel<PT, GSDR_ITEM_IBYTE>), dim3(nblocks, a->xm.q), dim3(PT::NT),
            a->lds_bytes, s, iq, stride, a->d_wipe, a->d_X, a->d_tw, plan_of<PT>(a), a->consumed, a->xm);
}

// The two-launch forward (acq_forward4_cols_kernel + acq_forward4_rows_kernel).
template <class PT>
void launch_forward_two(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, hipStream_t s)
{
    // the xm.q stored spectra per block (XMap): rows b * q + d, d < q
    const uint32_t nrows = nblocks * a->xm.q;
    const dim3 cg((PT::N2 + 255) / 256, nrows);
    if (item_type == GSDR_ITEM_GR_COMPLEX)
        hipLaunchKernelGGL((acq_forward4_cols_kernel<PT, GSDR_ITEM_GR_COMPLEX>), cg, dim3(256), 0, s, iq, stride,
            a->d_wipe, a->d_fscratch, a->d_tw, a->consumed, a->xm.q);
    else if (item_type == GSDR_ITEM_CSHORT)
        hipLaunchKernelGGL((acq_forward4_cols_kernel<PT, GSDR_ITEM_CSHORT>), cg, dim3(256), 0, s, iq, stride,
            a->d_wipe, a->d_fscratch, a->d_tw, a->consumed, a->xm.q);
    else
        hipLaunchKernelGGL((acq_forward4_cols_kernel<PT, GSDR_ITEM_IBYTE>), cg, dim3(256), 0, s, iq, stride,
            a->d_wipe, a->d_fscratch, a->d_tw, a->consumed, a->xm.q);
    hipLaunchKernelGGL((acq_forward4_rows_kernel<PT>), dim3(nrows * PT::R), dim3(PT::NT), PT::SubPlan::lds_bytes(), s,
        a->d_fscratch, a->d_X, a->d_tw_sub, nrows, a->xm.stride);
}

// General path (max_dwells > 1 and/or bit_transition_flag): forward spectra of
// all nblocks*K blocks, the dwell-accumulating correlate kernel, per-dwell
// statistics and the dwell decision.
template <class PT>
int launch_general(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, StageTimer& t)
{
    const size_t lds = a->lds_bytes;
    const uint32_t K = a->K;
    t.begin();
    launch_forward<PT>(a, iq, item_type, nblocks * K, stride, s);
    GSDR_HIP(hipGetLastError());
    t.end(0);
    AcqParams ap = params_of(a);
    t.begin();
    hipLaunchKernelGGL((acq_correlate_dwell_kernel<PT>), dim3(a->D * a->nprn * nblocks), dim3(PT::NT), lds, s, a->d_X,
        a->d_code_fft, a->d_stats, a->d_tw, plan_of<PT>(a), ap, a->d_acc, a->d_acc_slots, a->acc_words);
    GSDR_HIP(hipGetLastError());
    t.end(1);
    t.begin();
    hipLaunchKernelGGL(acq_reduce_dwell_kernel, dim3(nblocks * a->nprn), dim3(64), 0, s, a->d_stats, a->d_resk, res,
        a->d_prn, ap, stamp0, stride);
    GSDR_HIP(hipGetLastError());
    t.end(2);
    if (!ap.cfar)
        {
            t.begin();
            hipLaunchKernelGGL((acq_second_peak_dwell_kernel<PT>), dim3(K, nblocks * a->nprn), dim3(PT::NT), lds, s,
                a->d_X, a->d_code_fft, a->d_resk, a->d_tw, plan_of<PT>(a), ap, a->d_acc, a->d_acc_slots,
                a->acc_words);
            const uint32_t n = nblocks * a->nprn;
            hipLaunchKernelGGL(acq_decide_kernel, dim3((n + 255) / 256), dim3(256), 0, s, a->d_resk, res, K, n);
            GSDR_HIP(hipGetLastError());
            t.end(3);
        }
    return GSDR_OK;
}

// Split register four-step path (single dwell, with or without bit transition):
// forward spectra on PT, the split correlate's row maxima, the grid maximum, the
// selected row recomputed on PT for the first-maximum index / exact peak / CFAR
// power, and (peak ratio) the second peak on the same row.
template <class PT>
int launch_split_all(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, StageTimer& t)
{
    const size_t lds = a->lds_bytes;
    t.begin();
    if constexpr (requires_subplan<PT>::value)
        {
            if (a->d_fscratch)
                launch_forward_two<PT>(a, iq, item_type, nblocks, stride, s);
            else
                launch_forward<PT>(a, iq, item_type, nblocks, stride, s);
        }
    else
        launch_forward<PT>(a, iq, item_type, nblocks, stride, s);
    GSDR_HIP(hipGetLastError());
    t.end(0);
    AcqParams ap = params_of(a);
    t.begin();
    int rc = gsdr_acq_impl::launch_split(a, nblocks, s);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipGetLastError());
    t.end(1);
    t.begin();
    hipLaunchKernelGGL(acq_reduce_kernel, dim3(nblocks * a->nprn), dim3(64), 0, s, a->d_stats, res, a->d_prn, ap,
        stamp0, stride);
    GSDR_HIP(hipGetLastError());
    // the selected rows on the split plan itself (GSDR_ACQ_SPLIT_ARG=0: recomputed on PT);
    // CFAR with bit transition needs the opposite row's half window: recomputed on PT
    static const bool split_arg = !(std::getenv("GSDR_ACQ_SPLIT_ARG") && std::atoi(std::getenv("GSDR_ACQ_SPLIT_ARG")) == 0);
    if (split_arg && a->d_keys && !(ap.cfar && a->eff != a->N) && (ap.cfar || a->d_rowbuf))
        {
            int rc2 = gsdr_acq_impl::launch_split_argmax(a, nblocks, res, s);
            if (rc2 != GSDR_OK) return rc2;
        }
    else if (ap.cfar || !a->d_rowbuf)
        {
            hipLaunchKernelGGL((acq_argmax_four_kernel<PT>), dim3(nblocks * a->nprn), dim3(PT::NT), lds, s, a->d_X,
                a->d_code_fft, res, a->d_tw, plan_of<PT>(a), ap);
            GSDR_HIP(hipGetLastError());
        }
    else
        {
            // peak ratio: first and second peak from one recomputation of the row
            hipLaunchKernelGGL((acq_argmax_second_four_kernel<PT>), dim3(nblocks * a->nprn), dim3(PT::NT), lds, s,
                a->d_X, a->d_code_fft, res, a->d_tw, plan_of<PT>(a), ap, a->d_rowbuf);
            GSDR_HIP(hipGetLastError());
        }
    t.end(2);
    if (!ap.cfar && !a->d_rowbuf)
        {
            t.begin();
            hipLaunchKernelGGL((acq_second_peak_kernel<PT>), dim3(nblocks * a->nprn), dim3(PT::NT), lds, s, a->d_X,
                a->d_code_fft, res, a->d_tw, plan_of<PT>(a), ap);
            GSDR_HIP(hipGetLastError());
            t.end(3);
        }
    return GSDR_OK;
}

template <class PT>
int launch_all(gsdr_acq* a, const void* iq, int item_type, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s)
{
    const size_t lds = a->lds_bytes;
    StageTimer t(a, s);
    if constexpr (std::is_same<typename PT::PlanT, gsdr::fft::Plan4>::value)
        {
            if (a->split > 0) return launch_split_all<PT>(a, iq, item_type, nblocks, stride, stamp0, res, s, t);
        }
    if (a->general) return launch_general<PT>(a, iq, item_type, nblocks, stride, stamp0, res, s, t);
    t.begin();
    if (a->corr_variant > 0)
        {
            int rc = launch_forward_pk(a, iq, item_type, nblocks, stride, s);
            if (rc != GSDR_OK) return rc;
        }
    else
        launch_forward<PT>(a, iq, item_type, nblocks, stride, s);
    GSDR_HIP(hipGetLastError());
    t.end(0);
    t.begin();
    if (a->corr_variant > 0)
        {
            int rc = launch_corr_variant(a, nblocks, s);
            if (rc != GSDR_OK) return rc;
        }
    else
        {
            hipLaunchKernelGGL((acq_correlate_kernel<PT, false>), dim3(a->D * a->nprn, nblocks), dim3(PT::NT), lds, s,
                a->d_X, a->d_code_fft, a->d_stats, (float*)nullptr, a->d_tw, plan_of<PT>(a), a->D, a->nprn, 0u, a->xm);
        }
    GSDR_HIP(hipGetLastError());
    t.end(1);
    AcqParams ap = params_of(a);
    t.begin();
    hipLaunchKernelGGL(acq_reduce_kernel, dim3(nblocks * a->nprn), dim3(64), 0, s, a->d_stats, res, a->d_prn, ap,
        stamp0, stride);
    GSDR_HIP(hipGetLastError());
    if (a->corr_variant > 0 && a->corr_stat >= 1)
        {
            int rc = gsdr_acq_impl::launch_argmax_variant(a, nblocks, res, s);
            if (rc != GSDR_OK) return rc;
        }
    t.end(2);
    if (!ap.cfar)
        {
            t.begin();
            hipLaunchKernelGGL((acq_second_peak_kernel<PT>), dim3(nblocks * a->nprn), dim3(PT::NT), lds, s, a->d_X,
                a->d_code_fft, res, a->d_tw, plan_of<PT>(a), ap);
            GSDR_HIP(hipGetLastError());
            t.end(3);
        }
    return GSDR_OK;
}

// gsdr_acq_run_dwell: forward spectra of the block at a->d_iq, the accumulating
// grid kernel, the statistic with counter dwell+1 and (peak ratio) the second
// peak on the accumulated row.
template <class PT>
int launch_dwell(gsdr_acq* a, uint32_t dwell, uint64_t stamp, gsdr_acq_result* res, hipStream_t s)
{
    launch_forward<PT>(a, a->d_iq, a->conf.item_type, 1, a->consumed, s);
    GSDR_HIP(hipGetLastError());
    AcqParams ap = params_of(a);
    ap.counter = dwell + 1;
    hipLaunchKernelGGL((acq_dwell_grid_kernel<PT>), dim3(a->D * a->nprn), dim3(PT::NT), a->lds_bytes, s, a->d_X,
        a->d_code_fft, a->d_stats, a->d_tw, plan_of<PT>(a), ap, a->d_dgrid, dwell);
    GSDR_HIP(hipGetLastError());
    hipLaunchKernelGGL(acq_reduce_kernel, dim3(a->nprn), dim3(64), 0, s, a->d_stats, res, a->d_prn, ap, stamp,
        (uint64_t)a->consumed);
    GSDR_HIP(hipGetLastError());
    if (!ap.cfar)
        {
            hipLaunchKernelGGL(acq_grid_second_peak_kernel, dim3(a->nprn), dim3(256), 0, s, a->d_dgrid, res, ap);
            GSDR_HIP(hipGetLastError());
        }
    return GSDR_OK;
}

// aux: slot count in bits 0-15, first slot in bits 16+ (gsdr_acq_set_local_code
// transforms one slot, gsdr_acq_set_local_codes slots [0, nprn))
template <class PT>
int launch_code_fft(gsdr_acq* a, uint32_t aux)
{
    const uint32_t nprn = aux & 0xffffu, first = aux >> 16;
    hipLaunchKernelGGL((acq_code_fft_kernel<PT>), dim3(nprn), dim3(PT::NT), a->lds_bytes, a->stream,
        a->d_code_stage + (size_t)first * a->consumed, a->d_code_fft + (size_t)first * a->N, a->d_tw, plan_of<PT>(a),
        a->consumed, a->lead);
    GSDR_HIP(hipGetLastError());
    return GSDR_OK;
}

template <class PT>
int launch_dump(gsdr_acq* a, bool grid, uint32_t prn_slot)
{
    launch_forward<PT>(a, a->d_iq, a->conf.item_type, 1, a->consumed, a->stream);
    GSDR_HIP(hipGetLastError());
    if (grid)
        {
            hipLaunchKernelGGL((acq_correlate_kernel<PT, true>), dim3(a->D, 1), dim3(PT::NT), a->lds_bytes, a->stream,
                a->d_X, a->d_code_fft, a->d_stats, a->d_grid, a->d_tw, plan_of<PT>(a), a->D, a->nprn, prn_slot, a->xm);
            GSDR_HIP(hipGetLastError());
        }
    return GSDR_OK;
}


}  // namespace
