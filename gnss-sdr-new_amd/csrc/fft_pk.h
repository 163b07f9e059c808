// Packed-f32 LDS Stockham FFT for CDNA4 (gfx950).
//
// Same transform and data flow as fft_lds.h / fft_multi.h (unnormalised forward
// DFT, first stage from a load functor, last stage to a store functor, S-1 LDS
// round trips), but every complex value lives in one 64-bit VGPR pair and every
// complex operation is issued as packed-f32 VALU (v_pk_add_f32 / v_pk_mul_f32 /
// v_pk_fma_f32 with op_sel / neg modifiers):
//
//   complex add/sub            1 instruction   (scalar f32: 2)
//   p +- (-i)q                 1 instruction   (scalar: 2, plus the swap)
//   complex * complex          2 instructions  (scalar: 4)
//   real * complex (+ complex) 1 instruction   (scalar: 2)
//
// A wave64 v_pk_* instruction issues in the same 4 cycles as a v_add_f32, so
// the butterflies cost about half the VALU issue slots of the scalar form --
// the acquisition correlate kernel is VALU-issue-bound.
//
// The swizzled forms the compiler does not fold into op_sel/neg modifiers are
// written as inline asm; tools/pk_semantics.hip checks their semantics on the
// device.
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "fft_lds.h"
#include "fft_multi.h"

namespace gsdr
{
namespace pk
{

typedef float c2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ c2 from(float2 v) { return c2{v.x, v.y}; }
__device__ __forceinline__ float2 to(c2 v) { return make_float2(v.x, v.y); }

// a * b (complex)
__device__ __forceinline__ c2 mul(c2 a, c2 b)
{
    c2 r, o;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[1,0,0]"
        : "=v"(o)
        : "v"(a), "v"(b), "v"(r));
    return o;
}

// conj(a) * b
__device__ __forceinline__ c2 conj_mul(c2 a, c2 b)
{
    c2 r, o;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
    asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_hi:[1,0,0]"
        : "=v"(o)
        : "v"(a), "v"(b), "v"(r));
    return o;
}

// p + (-i) q = (p.x + q.y, p.y - q.x)
__device__ __forceinline__ c2 add_mi(c2 p, c2 q)
{
    c2 o;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(o) : "v"(p), "v"(q));
    return o;
}

// p - (-i) q = (p.x - q.y, p.y + q.x)
__device__ __forceinline__ c2 sub_mi(c2 p, c2 q)
{
    c2 o;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(o) : "v"(p), "v"(q));
    return o;
}

// (-i) a = (a.y, -a.x)
__device__ __forceinline__ c2 mul_mi(c2 a) { return a.yx * c2{1.0f, -1.0f}; }

// real scalar forms (the compiler emits one v_pk_mul / v_pk_fma with a broadcast operand)
__device__ __forceinline__ c2 scale(c2 a, float s) { return a * c2{s, s}; }
__device__ __forceinline__ c2 fmas(c2 a, float s, c2 c) { return __builtin_elementwise_fma(a, c2{s, s}, c); }

// a * w for a compile-time root w (special-cases 1, -1, +-i)
template <int M, int R>
__device__ __forceinline__ c2 mul_root(c2 a)
{
    constexpr int m = ((M % R) + R) % R;
    if constexpr (m == 0)
        return a;
    else if constexpr (4 * m == R)
        return mul_mi(a);
    else if constexpr (2 * m == R)
        return -a;
    else if constexpr (4 * m == 3 * R)
        return a.yx * c2{-1.0f, 1.0f};
    else
        {
            constexpr fft::Roots<R> W{};
            constexpr float wr = W.re[m], wi = W.im[m];
            // (a.x wr - a.y wi, a.y wr + a.x wi)
            const c2 t = a * c2{wr, wr};
            return __builtin_elementwise_fma(a.yx, c2{-wi, wi}, t);
        }
}

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F& f)
{
    if constexpr (B < E)
        {
            f(std::integral_constant<int, B>{});
            static_for<B + 1, E>(f);
        }
}

// ---- twiddle powers ----
// v[r] *= w1^r for r = 1 .. R-1 by one chain w <- w w1 (R-2 dependent complex
// products).  A baby-step / giant-step tree with a shorter dependency (r04e) was
// within noise at N = 4000 / 16000 / 32000 and 7 % slower on the 64000 split.
template <int R>
__device__ __forceinline__ void apply_powers(c2* v, c2 w1)
{
    c2 w = w1;
#pragma unroll
    for (int r = 1; r < R; ++r)
        {
            if (r > 1) w = mul(w, w1);
            v[r] = mul(v[r], w);
        }
}

// ---- small DFTs, natural order in and out, forward sign ----
template <int R>
struct Dft;

template <>
struct Dft<2>
{
    __device__ __forceinline__ static void run(c2* v)
    {
        const c2 a = v[0], b = v[1];
        v[0] = a + b;
        v[1] = a - b;
    }
};

template <>
struct Dft<3>
{
    __device__ __forceinline__ static void run(c2* v)
    {
        constexpr float h = 0.86602540378443864676f;  // sin(2pi/3)
        const c2 s = v[1] + v[2];
        const c2 d = v[1] - v[2];
        const c2 m = fmas(s, -0.5f, v[0]);
        const c2 t = scale(d, h);
        v[0] = v[0] + s;
        v[1] = add_mi(m, t);
        v[2] = sub_mi(m, t);
    }
};

template <>
struct Dft<4>
{
    __device__ __forceinline__ static void run(c2* v)
    {
        const c2 a = v[0] + v[2], b = v[0] - v[2];
        const c2 c = v[1] + v[3], d = v[1] - v[3];
        v[0] = a + c;
        v[2] = a - c;
        v[1] = add_mi(b, d);
        v[3] = sub_mi(b, d);
    }
};

template <>
struct Dft<5>
{
    __device__ __forceinline__ static void run(c2* v)
    {
        constexpr float c1 = 0.30901699437494742410f;   // cos(2pi/5)
        constexpr float c2_ = -0.80901699437494742410f;  // cos(4pi/5)
        constexpr float s1 = 0.95105651629515357212f;   // sin(2pi/5)
        constexpr float s2 = 0.58778525229247312917f;   // sin(4pi/5)
        const c2 a1 = v[1] + v[4], b1 = v[1] - v[4];
        const c2 a2 = v[2] + v[3], b2 = v[2] - v[3];
        const c2 x0 = v[0];
        const c2 p1 = fmas(a2, c2_, fmas(a1, c1, x0));
        const c2 p2 = fmas(a2, c1, fmas(a1, c2_, x0));
        const c2 q1 = fmas(b2, s2, scale(b1, s1));
        const c2 q2 = fmas(b2, -s1, scale(b1, s2));
        v[0] = x0 + a1 + a2;
        v[1] = add_mi(p1, q1);
        v[4] = sub_mi(p1, q1);
        v[2] = add_mi(p2, q2);
        v[3] = sub_mi(p2, q2);
    }
};

// Composite R = R1*R2 in registers: n = R2*n1 + n2, k = k1 + R1*k2.
template <int R1, int R2>
struct DftCT
{
    template <int N2, int K1>
    __device__ __forceinline__ static void twiddle(c2* t)
    {
        t[K1] = mul_root<N2 * K1, R1 * R2>(t[K1]);
        if constexpr (K1 + 1 < R1) twiddle<N2, K1 + 1>(t);
    }
    template <int N2>
    __device__ __forceinline__ static void cols(c2* v, c2* y)
    {
        c2 t[R1];
#pragma unroll
        for (int n1 = 0; n1 < R1; ++n1) t[n1] = v[R2 * n1 + N2];
        Dft<R1>::run(t);
        twiddle<N2, 0>(t);
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1) y[N2 * R1 + k1] = t[k1];
        if constexpr (N2 + 1 < R2) cols<N2 + 1>(v, y);
    }
    __device__ __forceinline__ static void run(c2* v)
    {
        c2 y[R1 * R2];
        cols<0>(v, y);
#pragma unroll
        for (int k1 = 0; k1 < R1; ++k1)
            {
                c2 t[R2];
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
template <>
struct Dft<32> : DftCT<4, 8>
{
};

// One Stockham stage over an N-point LDS buffer of c2.
//   TWP: inter-stage twiddles as powers of one table root (1 VMEM load per
//        butterfly, R-2 extra complex multiplies); else R-1 table loads.
//   ORD: the last stage hands each lane its outputs in increasing index order (a
//        first-maximum scan needs it); without ORD it visits butterfly by
//        butterfly, so a partially filled pass is skipped as a whole instead of
//        predicating every output (order-free reductions: max, sum).
// Measured and removed: twiddles from a per-stage table (-23 %)
// or an LDS copy of the middle stage's roots (-2.5 %), last-stage block padding
// (modelled conflicts removed, no gain), the barrier moved behind the butterflies
// or dropped before the last stage (within noise).
template <int R, int NT, int N, int Ns, bool TWP, bool FIRST, bool LAST, bool ORD, class Load, class Store, class Hook>
__device__ __forceinline__ void stage(c2* lds, const float2* __restrict__ tw, Load& load, Store& store, Hook& hook)
{
    constexpr int BPT = fft::bpt_for(R);
    constexpr int NB = N / R;
    constexpr int TSTRIDE = N / (Ns * R);
    c2 v[BPT][R];
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            // one pass per lane (BPT == 1): every lane loads, the idle ones from a
            // clamped in-bounds index -- no branch around the loads, so no
            // zero-filled registers for the idle lanes; their results are never
            // stored.  Several passes: the per-lane guard.
            const int j = (int)threadIdx.x + b * NT;
            if constexpr (BPT == 1 && NB % NT != 0)
                {
                    const int jj = min(j, NB - 1);
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        {
                            if constexpr (FIRST)
                                v[b][r] = load(b, r, jj + r * NB);
                            else
                                v[b][r] = lds[jj + r * NB];
                        }
                }
            else if (NB % NT == 0 || j < NB)
                {
#pragma unroll
                    for (int r = 0; r < R; ++r)
                        {
                            if constexpr (FIRST)
                                v[b][r] = load(b, r, j + r * NB);
                            else
                                v[b][r] = lds[j + r * NB];
                        }
                }
        }
    if constexpr (FIRST)
        hook();
    else
        __syncthreads();
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            const int j = (int)threadIdx.x + b * NT;
            if (NB % NT == 0 || j < NB)
                {
                    int k = 0;
                    if constexpr (!FIRST)
                        {
                            k = j % Ns;
                            const int step = k * TSTRIDE;
                            if constexpr (TWP)
                                apply_powers<R>(v[b], from(tw[step]));
                            else
                                {
#pragma unroll
                                    for (int r = 1; r < R; ++r) v[b][r] = mul(v[b][r], from(tw[r * step]));
                                }
                        }
                    Dft<R>::run(v[b]);
                    if constexpr (!LAST)
                        {
                            // block (j - k) R / (Ns R) = j / Ns of the last stage's input
                            const int base = (j - k) * R + k;
#pragma unroll
                            for (int r = 0; r < R; ++r) lds[base + r * Ns] = v[b][r];
                        }
                }
        }
    if constexpr (LAST && ORD)
        {
            // last stage: Ns = N/R and k = j, so output j + r*Ns; r outer, b inner
            // visits this lane's outputs in increasing index order, and the
            // compile-time slot r*BPT + b numbers them in that order
            static_assert(!LAST || Ns * R == N, "last stage");
#pragma unroll
            for (int r = 0; r < R; ++r)
                {
#pragma unroll
                    for (int b = 0; b < BPT; ++b)
                        {
                            const int j = (int)threadIdx.x + b * NT;
                            if (NB % NT == 0 || j < NB) store(j + r * Ns, v[b][r], r * BPT + b);
                        }
                }
        }
    else if constexpr (LAST)
        {
            static_assert(!LAST || Ns * R == N, "last stage");
#pragma unroll
            for (int b = 0; b < BPT; ++b)
                {
                    const int j = (int)threadIdx.x + b * NT;
                    if (NB % NT == 0 || j < NB)
                        {
#pragma unroll
                            for (int r = 0; r < R; ++r) store(j + r * Ns, v[b][r], r * BPT + b);
                        }
                }
        }
    else
        __syncthreads();
}

template <int NT, int N, int Ns, bool TWP, bool FIRST, bool ORD, int R, int... Rest, class Load, class Store, class Hook>
__device__ __forceinline__ void stages(c2* lds, const float2* __restrict__ tw, Load& load, Store& store, Hook& hook)
{
    constexpr bool LAST = sizeof...(Rest) == 0;
    stage<R, NT, N, Ns, TWP, FIRST, LAST, ORD>(lds, tw, load, store, hook);
    if constexpr (!LAST) stages<NT, N, Ns * R, TWP, false, ORD, Rest...>(lds, tw, load, store, hook);
}

// Compile-time packed plan.  load(b, r, i) -> c2 returns input element i
// (= j + r*N/R1 of this lane's b-th first-stage butterfly j); store(i, c2)
// consumes output element i, visited in increasing i per lane; hook() runs
// once the first stage's inputs are in registers (before its butterflies).
//   TWP: inter-stage twiddles as powers of one loaded root (1) or R-1 loads (0).
template <int NT_, int TWP_, int... Rs>
struct PkPlan
{
    static constexpr int NT = NT_;
    static constexpr bool TWP = TWP_ != 0;
    static constexpr int N = (Rs * ...);
    static constexpr int nstages = sizeof...(Rs);
    static constexpr int R1 = fft::FirstRadix<Rs...>::value;
    static constexpr int BPT1 = fft::bpt_for(R1);
    static constexpr int NB1 = N / R1;
    static constexpr size_t lds_bytes() { return (size_t)N * sizeof(c2); }
    // last stage: radix, butterflies per thread, output stride; store(i, v, slot)
    // receives slot = r*BPTL + b in [0, RL*BPTL), this lane's output order
    static constexpr int RL = (0, ..., Rs);
    static constexpr int BPTL = fft::bpt_for(RL);
    static constexpr int NSL = N / RL;
    static constexpr int NSLOTS = RL * BPTL;
    __device__ __forceinline__ static int index_of_slot(int slot)
    {
        return (int)threadIdx.x + (slot % BPTL) * NT + (slot / BPTL) * NSL;
    }
    template <bool ORD = true, class Load, class Store, class Hook>
    __device__ __forceinline__ static void run(c2* lds, const float2* __restrict__ tw, Load load, Store store, Hook hook)
    {
        stages<NT, N, 1, TWP, true, ORD, Rs...>(lds, tw, load, store, hook);
    }
};


}  // namespace pk
}  // namespace gsdr
