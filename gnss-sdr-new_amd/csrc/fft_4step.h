// Four-step FFT for transforms larger than one workgroup's LDS (N > 20352 points:
// Galileo E1 at 8 Msps = 32000, BeiDou/GPS at 25 Msps = 25000, Galileo at 25 Msps
// = 100000 -- configs C4/C5).
//
// N = R * N2 with a register radix R in {8,10,12,16,20,25} and an LDS-sized N2:
//   input index n = n1 + R*n2, output index k = k2 + N2*k1,
//   X[k2 + N2 k1] = sum_n1 W_R^{n1 k1} * ( W_N^{n1 k2} * sum_n2 x[n1 + R n2] W_N2^{n2 k2} ).
// One workgroup per transform (the same kernels as the LDS engine, through the
// plan-type interface PT::run(plan, lds, tw, load, store)):
//   phase 1: R LDS transforms of length N2 (stride-R input gather, L2-served),
//            each output scaled by the inter-step twiddle W_N^{n1 k2} (n1 k2 < N,
//            one table lookup) and written to the workgroup's global scratch row;
//   phase 2: every lane takes columns k2, loads the R values (coalesced across
//            lanes), runs the radix-R DFT in registers and hands X[k2 + N2 k1] to
//            the caller's store functor.
// The scratch rows (N complex each) come from a slot pool claimed with one atomic
// per transform, so any grid shape works with a bounded scratch allocation: a
// workgroup holds its slot only while it runs, so a free slot always appears.
#pragma once

#include "fft_lds.h"

namespace gsdr
{
namespace fft
{

struct Plan4
{
    int n;                        // N
    int r1;                       // register radix R
    Plan sub;                     // N2-point LDS plan (sub.n = N2)
    const float2* tw_sub;         // W_N2^m, m < N2
    float2* scratch;              // nslots rows of N complex
    uint32_t* slots;              // nslots/32 occupancy words (bit set = in use)
    int nwords;
};

inline int lds_elems(const Plan& p) { return p.n; }
inline int lds_elems(const Plan4& p) { return p.sub.n; }
__device__ __forceinline__ int lds_elems_dev(const Plan& p) { return p.n; }
__device__ __forceinline__ int lds_elems_dev(const Plan4& p) { return p.sub.n; }

template <int R, class Store>
__device__ __forceinline__ void four_step_columns(const Plan4& p, const float2* __restrict__ row, Store& store)
{
    const int N2 = p.sub.n;
    for (int k2 = (int)threadIdx.x; k2 < N2; k2 += (int)blockDim.x)
        {
            float2 v[R];
#pragma unroll
            for (int n1 = 0; n1 < R; ++n1) v[n1] = row[(size_t)n1 * N2 + k2];
            Dft<R>::run(v);
#pragma unroll
            for (int k1 = 0; k1 < R; ++k1) store(k2 + N2 * k1, v[k1]);
        }
}

template <int NT_>
struct FourStepPlan
{
    static constexpr int NT = NT_;
    static constexpr int N = 0;
    using PlanT = Plan4;
    // tw: W_N^m for m < N (the handle's full-size table)
    template <class Load, class Store>
    __device__ __forceinline__ static void run(const Plan4& p, float2* lds, const float2* __restrict__ tw, Load load,
        Store store)
    {
        __shared__ int s_slot;
        const int tid = (int)threadIdx.x;
        if (tid == 0)
            {
                int w = (int)((blockIdx.x + blockIdx.y * gridDim.x) % (unsigned)p.nwords);
                for (;;)
                    {
                        const uint32_t cur = __hip_atomic_load(&p.slots[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (cur != 0xffffffffu)
                            {
                                const int bit = __builtin_ctz(~cur);
                                const uint32_t old = __hip_atomic_fetch_or(&p.slots[w], 1u << bit, __ATOMIC_ACQUIRE,
                                    __HIP_MEMORY_SCOPE_AGENT);
                                if (!(old & (1u << bit)))
                                    {
                                        s_slot = w * 32 + bit;
                                        break;
                                    }
                            }
                        else
                            {
                                w = w + 1 == p.nwords ? 0 : w + 1;
                                __builtin_amdgcn_s_sleep(2);
                            }
                    }
            }
        __syncthreads();
        const int slot = s_slot;
        float2* row = p.scratch + (size_t)slot * p.n;
        const int N2 = p.sub.n;
        const int R = p.r1;
        for (int n1 = 0; n1 < R; ++n1)
            {
                auto ld = [&](int i) -> float2 { return load(n1 + R * i); };
                auto st = [&](int k2, float2 v) { row[(size_t)n1 * N2 + k2] = cmul(v, tw[n1 * k2]); };
                fft::run<NT>(p.sub, lds, p.tw_sub, ld, st);
            }
        __syncthreads();  // the workgroup's scratch row is complete (same CU, same L1)
        switch (R)
            {
            case 8: four_step_columns<8>(p, row, store); break;
            case 10: four_step_columns<10>(p, row, store); break;
            case 12: four_step_columns<12>(p, row, store); break;
            case 16: four_step_columns<16>(p, row, store); break;
            case 20: four_step_columns<20>(p, row, store); break;
            case 25: four_step_columns<25>(p, row, store); break;
            default: break;
            }
        __syncthreads();  // every lane's reads of the row have returned
        if (tid == 0)
            __hip_atomic_fetch_and(&p.slots[slot >> 5], ~(1u << (slot & 31)), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
};

}  // namespace fft
}  // namespace gsdr
