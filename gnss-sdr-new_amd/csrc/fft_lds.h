// Mixed-radix Stockham FFT held in one workgroup's LDS, for CDNA4 (gfx950).
//
// Used by the acquisition kernels for the D forward transforms of the wiped-off
// input and, fused with the code product, |.|^2 and the row reductions, for the
// P*D correlation transforms (pcps_acquisition.cc:655-686).  Unnormalised
// forward transform, exp(-2*pi*i*n*k/N), like FFTW's forward plan; the inverse
// transform of the reference is obtained as conj(FFT(conj(.))), which leaves
// |.|^2 unchanged so the fused kernel never conjugates the output.
//
// Structure of one radix-R stage (Ns = product of the radices already applied):
//   butterfly j in [0, N/R): inputs  x[j + r*N/R], r = 0..R-1
//                            twiddle x_r *= W_{Ns*R}^{r*(j mod Ns)}
//                            outputs y[(j - j mod Ns)*R + j mod Ns + r*Ns]
// The first stage reads straight from a caller functor (global memory, coalesced
// in j) and the last stage hands its outputs to a caller functor in registers
// (coalesced stores or a fused reduction), so an S-stage transform makes S-1
// LDS round trips.  Every thread stages its butterfly inputs in VGPRs before the
// barrier, so each stage runs in place in a single N-point LDS buffer.
#pragma once

#include <hip/hip_runtime.h>

namespace gsdr
{
namespace fft
{

constexpr int kMaxStages = 8;
constexpr int kElemBudget = 16;  // complex values per thread per stage (VGPR budget)

struct Plan
{
    int n;
    int nstages;
    int radix[kMaxStages];
};

constexpr int bpt_for(int R) { return (kElemBudget + R - 1) / R; }

// ---- compile-time roots of unity (constant-folded into the butterflies) ----
constexpr double kPi = 3.141592653589793238462643383279502884;
constexpr double ct_wrap(double x)
{
    while (x > kPi) x -= 2.0 * kPi;
    while (x < -kPi) x += 2.0 * kPi;
    return x;
}
constexpr double ct_sin(double x)
{
    x = ct_wrap(x);
    double term = x, sum = x;
    for (int k = 1; k < 24; ++k)
        {
            term *= -x * x / (double)((2 * k) * (2 * k + 1));
            sum += term;
        }
    return sum;
}
constexpr double ct_cos(double x) { return ct_sin(x + kPi / 2.0); }

template <int R>
struct Roots
{
    float re[R];
    float im[R];
    constexpr Roots() : re(), im()
    {
        for (int m = 0; m < R; ++m)
            {
                re[m] = (float)ct_cos(2.0 * kPi * m / R);
                im[m] = (float)(-ct_sin(2.0 * kPi * m / R));
            }
    }
};

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }
__device__ __forceinline__ float2 mul_neg_i(float2 a) { return make_float2(a.y, -a.x); }  // -i*a

// ---- small DFTs, natural order in and out, forward sign ----
template <int R>
struct Dft;

template <>
struct Dft<2>
{
    __device__ __forceinline__ static void run(float2* v)
    {
        float2 a = v[0], b = v[1];
        v[0] = cadd(a, b);
        v[1] = csub(a, b);
    }
};

template <>
struct Dft<3>
{
    __device__ __forceinline__ static void run(float2* v)
    {
        constexpr float h = 0.86602540378443864676f;  // sin(2pi/3)
        float2 s = cadd(v[1], v[2]);
        float2 d = csub(v[1], v[2]);
        float2 m = make_float2(v[0].x - 0.5f * s.x, v[0].y - 0.5f * s.y);
        float2 t = mul_neg_i(cscale(d, h));
        v[0] = cadd(v[0], s);
        v[1] = cadd(m, t);
        v[2] = csub(m, t);
    }
};

template <>
struct Dft<4>
{
    __device__ __forceinline__ static void run(float2* v)
    {
        float2 a = cadd(v[0], v[2]), b = csub(v[0], v[2]);
        float2 c = cadd(v[1], v[3]), d = mul_neg_i(csub(v[1], v[3]));
        v[0] = cadd(a, c);
        v[2] = csub(a, c);
        v[1] = cadd(b, d);
        v[3] = csub(b, d);
    }
};

template <>
struct Dft<5>
{
    __device__ __forceinline__ static void run(float2* v)
    {
        constexpr float c1 = 0.30901699437494742410f;   // cos(2pi/5)
        constexpr float c2 = -0.80901699437494742410f;  // cos(4pi/5)
        constexpr float s1 = 0.95105651629515357212f;   // sin(2pi/5)
        constexpr float s2 = 0.58778525229247312917f;   // sin(4pi/5)
        float2 a1 = cadd(v[1], v[4]), b1 = csub(v[1], v[4]);
        float2 a2 = cadd(v[2], v[3]), b2 = csub(v[2], v[3]);
        float2 x0 = v[0];
        float2 p1 = make_float2(x0.x + c1 * a1.x + c2 * a2.x, x0.y + c1 * a1.y + c2 * a2.y);
        float2 p2 = make_float2(x0.x + c2 * a1.x + c1 * a2.x, x0.y + c2 * a1.y + c1 * a2.y);
        float2 q1 = mul_neg_i(make_float2(s1 * b1.x + s2 * b2.x, s1 * b1.y + s2 * b2.y));
        float2 q2 = mul_neg_i(make_float2(s2 * b1.x - s1 * b2.x, s2 * b1.y - s1 * b2.y));
        v[0] = make_float2(x0.x + a1.x + a2.x, x0.y + a1.y + a2.y);
        v[1] = cadd(p1, q1);
        v[4] = csub(p1, q1);
        v[2] = cadd(p2, q2);
        v[3] = csub(p2, q2);
    }
};

// Composite R = R1*R2 in registers: n = R2*n1 + n2, k = k1 + R1*k2.
template <int R1, int R2>
struct DftCT
{
    __device__ __forceinline__ static void run(float2* v)
    {
        constexpr int R = R1 * R2;
        constexpr Roots<R> W{};
        float2 y[R];
#pragma unroll
        for (int n2 = 0; n2 < R2; ++n2)
            {
                float2 t[R1];
#pragma unroll
                for (int n1 = 0; n1 < R1; ++n1) t[n1] = v[R2 * n1 + n2];
                Dft<R1>::run(t);
#pragma unroll
                for (int k1 = 0; k1 < R1; ++k1)
                    {
                        const int m = (n2 * k1) % R;
                        y[n2 * R1 + k1] = (m == 0) ? t[k1] : cmul(t[k1], make_float2(W.re[m], W.im[m]));
                    }
            }
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1)
            {
                float2 t[R2];
#pragma unroll
                for (int n2 = 0; n2 < R2; ++n2) t[n2] = y[n2 * R1 + k1];
                Dft<R2>::run(t);
#pragma unroll
                for (int k2 = 0; k2 < R2; ++k2) v[k1 + R1 * k2] = t[k2];
            }
    }
};

template <>
struct Dft<6> : DftCT<2, 3>
{
};
template <>
struct Dft<8> : DftCT<2, 4>
{
};
template <>
struct Dft<10> : DftCT<2, 5>
{
};
template <>
struct Dft<12> : DftCT<4, 3>
{
};
template <>
struct Dft<16> : DftCT<4, 4>
{
};
template <>
struct Dft<20> : DftCT<4, 5>
{
};
template <>
struct Dft<25> : DftCT<5, 5>
{
};

// One Stockham stage.  lds: N complex.  tw: W_N^m, m in [0, N) (global, L2-resident).
// FIRST: inputs come from load(); LAST: outputs go to store().  Both are
// compile-time so no lane ever issues the alternative memory operation.
template <int R, int NT, bool FIRST, bool LAST, class Load, class Store>
__device__ __forceinline__ void stage(float2* lds, const float2* __restrict__ tw, int N, int Ns, Load& load,
    Store& store)
{
    constexpr int BPT = bpt_for(R);
    const int nb = N / R;
    const int tstride = N / (Ns * R);
    float2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            const int j = (int)threadIdx.x + b * NT;
            if (j < nb)
                {
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        {
                            if constexpr (FIRST)
                                v[b][r] = load(j + r * nb);
                            else
                                v[b][r] = lds[j + r * nb];
                        }
                }
        }
    if constexpr (!FIRST) __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            const int j = (int)threadIdx.x + b * NT;
            if (j < nb)
                {
                    int k = 0;
                    if constexpr (!FIRST)
                        {
                            k = j % Ns;
                            const int step = k * tstride;
#pragma unroll
                            for (int r = 1; r < R; ++r) v[b][r] = cmul(v[b][r], tw[r * step]);
                        }
                    Dft<R>::run(v[b]);
                    const int base = (j - k) * R + k;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        {
                            const int o = base + r * Ns;
                            if constexpr (LAST)
                                store(o, v[b][r]);
                            else
                                lds[o] = v[b][r];
                        }
                }
        }
    if constexpr (!LAST) __syncthreads();
}

template <int NT, bool FIRST, bool LAST, class Load, class Store>
__device__ __forceinline__ void stage_dispatch(int R, float2* lds, const float2* __restrict__ tw, int N, int Ns,
    Load& load, Store& store)
{
    switch (R)
        {
        case 2: stage<2, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 3: stage<3, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 4: stage<4, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 5: stage<5, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 6: stage<6, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 8: stage<8, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 10: stage<10, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 12: stage<12, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 16: stage<16, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 20: stage<20, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        case 25: stage<25, NT, FIRST, LAST>(lds, tw, N, Ns, load, store); break;
        default: break;
        }
}

// Run a runtime plan (>= 2 stages): the generic fallback for sizes without a
// compile-time plan.  The caller must have synchronised the workgroup if the LDS
// buffer was in use before the call.  load(i) returns input element i; store(i, v)
// consumes output element i (natural-order index).
template <int NT, class Load, class Store>
__device__ __forceinline__ void run(const Plan& p, float2* lds, const float2* __restrict__ tw, Load load,
    Store store)
{
    stage_dispatch<NT, true, false>(p.radix[0], lds, tw, p.n, 1, load, store);
    int Ns = p.radix[0];
    for (int s = 1; s < p.nstages - 1; ++s)
        {
            stage_dispatch<NT, false, false>(p.radix[s], lds, tw, p.n, Ns, load, store);
            Ns *= p.radix[s];
        }
    stage_dispatch<NT, false, true>(p.radix[p.nstages - 1], lds, tw, p.n, Ns, load, store);
}

// Compile-time plan: N, Ns and the twiddle strides are constants, so the index
// arithmetic folds and each kernel's VGPR budget is that of its largest radix.
template <int NT, int N, int Ns, bool FIRST, int R, int... Rest, class Load, class Store>
__device__ __forceinline__ void static_stages(float2* lds, const float2* __restrict__ tw, Load& load, Store& store)
{
    constexpr bool LAST = sizeof...(Rest) == 0;
    stage<R, NT, FIRST, LAST>(lds, tw, N, Ns, load, store);
    if constexpr (!LAST) static_stages<NT, N, Ns * R, false, Rest...>(lds, tw, load, store);
}

template <int NT_, int... Rs>
struct StaticPlan
{
    static constexpr int NT = NT_;
    static constexpr int N = (Rs * ...);
    static constexpr int nstages = sizeof...(Rs);
    using PlanT = Plan;
    template <class Load, class Store>
    __device__ __forceinline__ static void run(const Plan&, float2* lds, const float2* __restrict__ tw, Load load,
        Store store)
    {
        static_stages<NT, N, 1, true, Rs...>(lds, tw, load, store);
    }
    static Plan plan()
    {
        Plan p{};
        p.n = N;
        p.nstages = nstages;
        const int r[] = {Rs...};
        for (int i = 0; i < kMaxStages; ++i) p.radix[i] = i < nstages ? r[i] : 1;
        return p;
    }
};

template <int NT_>
struct RuntimePlan
{
    static constexpr int NT = NT_;
    static constexpr int N = 0;
    using PlanT = Plan;
    template <class Load, class Store>
    __device__ __forceinline__ static void run(const Plan& p, float2* lds, const float2* __restrict__ tw, Load load,
        Store store)
    {
        fft::run<NT>(p, lds, tw, load, store);
    }
};

}  // namespace fft
}  // namespace gsdr
