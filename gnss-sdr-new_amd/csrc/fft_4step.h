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
#include "fft_pk.h"

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

// Claim a scratch row from the slot pool (one atomic per transform; a workgroup
// holds its slot only while it runs, so a free slot always appears).
__device__ __forceinline__ int four_step_claim(const Plan4& p)
{
    __shared__ int s_slot;
    if (threadIdx.x == 0)
        {
            int w = (int)((blockIdx.x + blockIdx.y * gridDim.x) % (unsigned)p.nwords);
            for (;;)
                {
                    const uint32_t cur = __hip_atomic_load(&p.slots[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (cur != 0xffffffffu)
                        {
                            const int bit = __builtin_ctz(~cur);
                            const uint32_t old =
                                __hip_atomic_fetch_or(&p.slots[w], 1u << bit, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
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
    return s_slot;
}

// Inter-step twiddles W_N^{n2 k1}, k1 = 1..R-1, of column n2: the table roots
// b_i = W_N^{n2 2^i} -- a few reads whose lane addresses stride 2^i entries,
// instead of R-1 reads striding up to R-1 entries (up to 64 cache lines per
// wave-instruction) -- and W_N^{n2 k1} as the product of the b_i of k1's set bits
// (at most three multiplies, fp32 error a few ulp).  Computed per k1 right before
// its use, so only the bases stay live.
template <int R>
struct ColTwiddles
{
    static constexpr int NBASE = R > 16 ? 5 : (R > 8 ? 4 : (R > 4 ? 3 : 2));
    pk::c2 b[NBASE];
    __device__ __forceinline__ ColTwiddles(const float2* __restrict__ tw, int n2)
    {
#pragma unroll
        for (int i = 0; i < NBASE; ++i)
            if ((1 << i) < R) b[i] = pk::from(tw[n2 << i]);
    }
    __device__ __forceinline__ pk::c2 operator()(int k) const
    {
        pk::c2 w{1.0f, 0.0f};
        bool first = true;
#pragma unroll
        for (int i = 0; i < NBASE; ++i)
            if (k & (1 << i))
                {
                    w = first ? b[i] : pk::mul(w, b[i]);
                    first = false;
                }
        return w;
    }
};

// Four-step on the packed-f32 engine (fft_pk.h): N = R * SP::N with compile-time R
// and sub-plan SP (e.g. 64000 = 16 x 4000, 100000 = 25 x 4000, 25000 = 5 x 5000).
// Same decomposition and data flow as FourStepPlan (decimation in frequency,
// X[k1 + R k2] = sum_n2 W_N2^{n2 k2} (W_N^{n2 k1} sum_n1 x[n1 N2 + n2] W_R^{n1 k1})),
// with the column DFT as packed butterflies and the R sub-transforms on the
// packed Stockham plan; outputs reach the caller's store functor in no particular
// order (every consumer reduces with an index tie-break or stores by index).
template <int R_, class SP, bool PF = true>
struct FourStepPkPlan
{
    static constexpr int NT = SP::NT;
    static constexpr int R = R_;
    static constexpr int N2 = SP::N;
    static constexpr int N = R * N2;
    using PlanT = Plan4;
    using SubPlan = SP;
    // tw: W_N^m for m < N (the handle's full-size table); p.tw_sub: W_N2^m, m < N2
    template <class Load, class Store>
    __device__ __forceinline__ static void run(const Plan4& p, float2* lds, const float2* __restrict__ tw, Load load,
        Store store)
    {
        using pk::c2;
        const int slot = four_step_claim(p);
        c2* row = reinterpret_cast<c2*>(p.scratch) + (size_t)slot * N;
        // phase 1: columns n2 -- R coalesced loads, packed DFT_R, inter-step twiddle
        // W_N^{n2 k1} (one table read each, n2 k1 < N), row k1 of the scratch
        for (int n2 = (int)threadIdx.x; n2 < N2; n2 += NT)
            {
                c2 v[R];
#pragma unroll
                for (int n1 = 0; n1 < R; ++n1) v[n1] = pk::from(load(n1 * N2 + n2));
                pk::Dft<R>::run(v);
                const ColTwiddles<R> w(tw, n2);
                row[n2] = v[0];
#pragma unroll
                for (int k1 = 1; k1 < R; ++k1) row[(size_t)k1 * N2 + n2] = pk::mul(v[k1], w(k1));
            }
        __syncthreads();  // the workgroup's scratch row is complete (same CU, same L1)
        // phase 2: the R sub-transforms; the first-stage inputs of row k1 + 1 are
        // fetched into registers while row k1's butterflies run (the plan's hook),
        // so the scratch reads overlap compute instead of stalling each transform
        constexpr int R1 = SP::R1, BPT1 = SP::BPT1, NB1 = SP::NB1;
        c2 pre[BPT1][R1];
        auto fetch = [&](int k1) {
            const c2* rk = row + (size_t)k1 * N2;
#pragma unroll
            for (int bb = 0; bb < BPT1; ++bb)
                {
                    const int j = (int)threadIdx.x + bb * NT;
                    const int j0 = (int)(threadIdx.x & ~63u) + bb * NT;
                    if (NB1 % NT == 0 || j0 < NB1)
                        {
                            const int jj = min(j, NB1 - 1);
#pragma unroll
                            for (int r = 0; r < R1; ++r) pre[bb][r] = rk[jj + r * NB1];
                        }
                }
        };
        fetch(0);
        c2* l = reinterpret_cast<c2*>(lds);
        if constexpr (!PF)
            {
                // no prefetch: each sub-transform reads its row in its first stage
                for (int k1 = 0; k1 < R; ++k1)
                    {
                        const c2* rk = row + (size_t)k1 * N2;
                        auto ld = [&](int, int, int i) -> c2 { return rk[i]; };
                        auto st = [&](int k2, c2 v, int) { store(k1 + R * k2, pk::to(v)); };
                        SP::template run<false>(l, p.tw_sub, ld, st, [] {});
                        __syncthreads();
                    }
                if (threadIdx.x == 0)
                    __hip_atomic_fetch_and(&p.slots[slot >> 5], ~(1u << (slot & 31)), __ATOMIC_RELEASE,
                        __HIP_MEMORY_SCOPE_AGENT);
                return;
            }
        for (int k1 = 0; k1 < R; ++k1)
            {
                c2 cur[BPT1][R1];  // (PF only)
#pragma unroll
                for (int bb = 0; bb < BPT1; ++bb)
#pragma unroll
                    for (int r = 0; r < R1; ++r) cur[bb][r] = pre[bb][r];
                auto ld = [&](int bb, int r, int) -> c2 { return cur[bb][r]; };
                auto st = [&](int k2, c2 v, int) { store(k1 + R * k2, pk::to(v)); };
                auto hook = [&]() {
                    if (PF && k1 + 1 < R) fetch(k1 + 1);
                };
                SP::template run<false>(l, p.tw_sub, ld, st, hook);
                __syncthreads();  // the LDS buffer is reused by the next sub-transform
            }
        if (threadIdx.x == 0)
            __hip_atomic_fetch_and(&p.slots[slot >> 5], ~(1u << (slot & 31)), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
};

}  // namespace fft
}  // namespace gsdr
