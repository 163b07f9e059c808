// Multi-transform LDS Stockham FFT: PB independent N-point transforms per
// workgroup, advanced in lock-step so every lane carries PB butterflies of the
// same (stage, j): the input loads a caller can share (the spectrum X_{b,d} in
// the acquisition correlate kernel) and every inter-stage twiddle are loaded once
// and applied PB times, and the PB dependency chains interleave (ILP).
//
// Optional LDS padding: transform t, element i lives at lds[t*STRIDE + i + i/32],
// which spreads the stride-R writes of the first stage over the banks.
#pragma once

#include "fft_lds.h"

namespace gsdr
{
namespace fft
{

template <bool PAD>
__device__ __forceinline__ int phys(int i)
{
    return PAD ? i + (i >> 5) : i;
}

template <int R, int NT, int PB, bool PAD, bool TWP, bool FIRST, bool LAST, class Load, class Store, class Hook>
__device__ __forceinline__ void mstage(float2* lds, int stride, const float2* __restrict__ tw, int N, int Ns,
    Load& load, Store& store, Hook& hook)
{
    constexpr int BPT = bpt_for(R);
    const int nb = N / R;
    const int tstride = N / (Ns * R);
    float2 v[PB][BPT][R];
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
                                {
                                    float2 col[PB];
                                    load(b, r, j + r * nb, col);
#pragma unroll
                                    for (int t = 0; t < PB; ++t) v[t][b][r] = col[t];
                                }
                            else
                                {
                                    const int a = phys<PAD>(j + r * nb);
#pragma unroll
                                    for (int t = 0; t < PB; ++t) v[t][b][r] = lds[t * stride + a];
                                }
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
                            if constexpr (TWP)
                                {
                                    // one table load, the other twiddles as powers (error ~ r ulp)
                                    const float2 w1 = tw[step];
                                    float2 w = w1;
#pragma unroll
                                    for (int r = 1; r < R; ++r)
                                        {
                                            if (r > 1) w = cmul(w, w1);
#pragma unroll
                                            for (int t = 0; t < PB; ++t) v[t][b][r] = cmul(v[t][b][r], w);
                                        }
                                }
                            else
                                {
#pragma unroll
                                    for (int r = 1; r < R; ++r)
                                        {
                                            const float2 w = tw[r * step];
#pragma unroll
                                            for (int t = 0; t < PB; ++t) v[t][b][r] = cmul(v[t][b][r], w);
                                        }
                                }
                        }
#pragma unroll
                    for (int t = 0; t < PB; ++t) Dft<R>::run(v[t][b]);
                    const int base = (j - k) * R + k;
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        {
                            const int o = base + r * Ns;
                            if constexpr (LAST)
                                {
                                    float2 col[PB];
#pragma unroll
                                    for (int t = 0; t < PB; ++t) col[t] = v[t][b][r];
                                    store(o, col);
                                }
                            else
                                {
                                    const int a = phys<PAD>(o);
#pragma unroll
                                    for (int t = 0; t < PB; ++t) lds[t * stride + a] = v[t][b][r];
                                }
                        }
                }
        }
    // the first stage's inputs are dead: let the caller start its next loads now
    if constexpr (FIRST) hook();
    if constexpr (!LAST) __syncthreads();
}

template <int NT, int PB, bool PAD, bool TWP, int N, int Ns, bool FIRST, int R, int... Rest, class Load, class Store,
    class Hook>
__device__ __forceinline__ void static_mstages(float2* lds, int stride, const float2* __restrict__ tw, Load& load,
    Store& store, Hook& hook)
{
    constexpr bool LAST = sizeof...(Rest) == 0;
    mstage<R, NT, PB, PAD, TWP, FIRST, LAST>(lds, stride, tw, N, Ns, load, store, hook);
    if constexpr (!LAST)
        static_mstages<NT, PB, PAD, TWP, N, Ns * R, false, Rest...>(lds, stride, tw, load, store, hook);
}

template <int R, int... Rest>
struct FirstRadix
{
    static constexpr int value = R;
};

// second radix of a plan (0 for a one-stage plan)
template <int... Rs>
struct SecondRadix
{
    static constexpr int value = 0;
};
template <int R1, int R2, int... Rest>
struct SecondRadix<R1, R2, Rest...>
{
    static constexpr int value = R2;
};

// Compile-time multi-transform plan.  load(b, r, i, float2 (&)[PB]) fills element
// i (= j + r*N/R1 of this lane's b-th first-stage butterfly j) of the PB inputs;
// store(i, const float2 (&)[PB]) consumes output element i; hook() runs once the
// first stage has consumed its inputs.
// TWP: inter-stage twiddles by powers of one loaded root (fewer VMEM loads).
template <int NT_, int PB_, bool PAD_, bool TWP_, int... Rs>
struct MultiPlan
{
    static constexpr int NT = NT_;
    static constexpr int PB = PB_;
    static constexpr bool PAD = PAD_;
    static constexpr bool TWP = TWP_;
    static constexpr int N = (Rs * ...);
    static constexpr int nstages = sizeof...(Rs);
    // per-transform LDS stride in complex elements (even, so float4 alignment holds)
    static constexpr int STRIDE = PAD ? ((N + (N >> 5) + 2) & ~1) : N;
    static constexpr int R1 = FirstRadix<Rs...>::value;
    static constexpr int BPT1 = bpt_for(R1);
    static constexpr int NB1 = N / R1;
    static constexpr size_t lds_bytes() { return (size_t)PB * STRIDE * sizeof(float2); }
    template <class Load, class Store, class Hook>
    __device__ __forceinline__ static void run(float2* lds, const float2* __restrict__ tw, Load load, Store store,
        Hook hook)
    {
        static_mstages<NT, PB, PAD, TWP, N, 1, true, Rs...>(lds, STRIDE, tw, load, store, hook);
    }
    template <class Load, class Store>
    __device__ __forceinline__ static void run(float2* lds, const float2* __restrict__ tw, Load load, Store store)
    {
        run(lds, tw, load, store, [] {});
    }
};

}  // namespace fft
}  // namespace gsdr
