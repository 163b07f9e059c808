// Four-step FFT for transforms larger than one workgroup's LDS (N > 20352 points:
// Galileo E1 at 8 Msps = 32000, BeiDou/GPS at 25 Msps = 25000, Galileo at 25 Msps
// = 100000 -- configs C4/C5).
//
// N = R * N2 with a register radix R in {8,10,12,16,20,25} and an LDS-sized N2,
// decimation in frequency:
//   input index n = n1*N2 + n2, output index k = k1 + R*k2,
//   X[k1 + R k2] = sum_n2 W_N2^{n2 k2} ( W_N^{n2 k1} * sum_n1 x[n1 N2 + n2] W_R^{n1 k1} ).
// One workgroup per transform (the same kernels as the LDS engine, through the
// plan-type interface PT::run(plan, lds, tw, load, store)):
//   phase 1: every lane takes columns n2, loads x[n1 N2 + n2] for the R values of
//            n1 (coalesced across lanes, each input read once), runs the radix-R
//            DFT in registers, scales by the twiddle W_N^{n2 k1} (n2 k1 < N, one
//            table lookup) and writes row k1 of the workgroup's global scratch
//            (coalesced);
//   phase 2: R LDS transforms of length N2 over the scratch rows, handing
//            X[k1 + R k2] to the caller's store functor.
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

template <int R, class Load>
__device__ __forceinline__ void four_step_columns(const Plan4& p, float2* __restrict__ row,
    const float2* __restrict__ tw, Load& load)
{
    const int N2 = p.sub.n;
    for (int n2 = (int)threadIdx.x; n2 < N2; n2 += (int)blockDim.x)
        {
            float2 v[R];
#pragma unroll
            for (int n1 = 0; n1 < R; ++n1) v[n1] = load(n1 * N2 + n2);
            Dft<R>::run(v);
#pragma unroll
            for (int k1 = 0; k1 < R; ++k1) row[(size_t)k1 * N2 + n2] = k1 == 0 ? v[0] : cmul(v[k1], tw[n2 * k1]);
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
        switch (R)
            {
            case 8: four_step_columns<8>(p, row, tw, load); break;
            case 10: four_step_columns<10>(p, row, tw, load); break;
            case 12: four_step_columns<12>(p, row, tw, load); break;
            case 16: four_step_columns<16>(p, row, tw, load); break;
            case 20: four_step_columns<20>(p, row, tw, load); break;
            case 25: four_step_columns<25>(p, row, tw, load); break;
            default: break;
            }
        __syncthreads();  // the workgroup's scratch row is complete (same CU, same L1)
        for (int k1 = 0; k1 < R; ++k1)
            {
                const float2* rk = row + (size_t)k1 * N2;
                auto ld = [&](int i) -> float2 { return rk[i]; };
                auto st = [&](int k2, float2 v) { store(k1 + R * k2, v); };
                fft::run<NT>(p.sub, lds, p.tw_sub, ld, st);
            }
        __syncthreads();  // every lane's reads of the row have returned
        if (tid == 0)
            __hip_atomic_fetch_and(&p.slots[slot >> 5], ~(1u << (slot & 31)), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
};

}  // namespace fft
}  // namespace gsdr
