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
// v[r] *= w1^r for r = 1 .. R-1.  GSDR_TW_TREE 0: one chain w <- w w1 (R-2
// dependent complex products); 1: baby-step / giant-step -- the powers w^1 .. w^(S-1)
// and the giants w^(S a), then w^(S a + b) = w^(S a) w^b -- the same R-2 products
// with a dependency depth of about log2(S) + R/S instead of R-2.  Measured in r04e:
// within noise at N = 4000 / 16000 / 32000, 7 % slower on the 64000 split (register
// pressure), so off.
#ifndef GSDR_TW_TREE
#define GSDR_TW_TREE 0
#endif
template <int R>
__device__ __forceinline__ void apply_powers(c2* v, c2 w1)
{
    if constexpr (R <= 2 || !GSDR_TW_TREE)
        {
            c2 w = w1;
#pragma unroll
            for (int r = 1; r < R; ++r)
                {
                    if (r > 1) w = mul(w, w1);
                    v[r] = mul(v[r], w);
                }
        }
    else
        {
            constexpr int S = R >= 32 ? 8 : (R % 5 == 0 ? 5 : 4);
            c2 b[S];  // b[k] = w^k, k < S
            b[1] = w1;
#pragma unroll
            for (int k = 2; k < S; ++k) b[k] = mul(b[k / 2], b[k - k / 2]);
            const c2 g1 = mul(b[S / 2], b[S - S / 2]);  // w^S
            c2 g = g1;
#pragma unroll
            for (int r = 1; r < R; ++r)
                {
                    const int a = r / S, k = r % S;
                    if (a > 1 && k == 0) g = mul(g, g1);  // w^(S a)
                    if (a == 0)
                        v[r] = mul(v[r], b[k]);
                    else if (k == 0)
                        v[r] = mul(v[r], g);
                    else
                        v[r] = mul(v[r], mul(g, b[k]));
                }
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

// ---- per-stage twiddle table (TWP == 2) ----
// Row length for a radix-R stage: the R-1 roots, padded to an even count.
constexpr int stage_tw_row(int R) { return (R - 1 + 1) & ~1; }
// LDS copy of the middle stage's table (TWP == 3): rows of stage_tw_row(R) + 2
// entries, so 16 lanes reading 16 different rows with ds_read_b128 hit 16
// different bank quads (row stride 36 dwords for R = 16).
constexpr int lds_tw_row(int R) { return stage_tw_row(R) + 2; }

template <int... Rs>
constexpr size_t stage_tw_entries()
{
    constexpr int r[] = {Rs...};
    size_t n = 0;
    int ns = r[0];
    for (size_t s = 1; s < sizeof...(Rs); ++s)
        {
            n += (size_t)ns * stage_tw_row(r[s]);
            ns *= r[s];
        }
    return n;
}

// Host: entries N, N+1, ... of the table the kernels read: for every non-first
// stage s (radix R, Ns-point sub-transforms, TSTRIDE = N/(Ns R)) and k < Ns the
// row W_N^{r k TSTRIDE}, r = 1..R-1 (angles in double, rounded once).
template <int... Rs>
inline void stage_tw_fill(float2* tw, int N)
{
    constexpr int r[] = {Rs...};
    size_t o = (size_t)N;
    int ns = r[0];
    for (size_t s = 1; s < sizeof...(Rs); ++s)
        {
            const int R = r[s], row = stage_tw_row(R), ts = N / (ns * R);
            for (int k = 0; k < ns; ++k)
                for (int q = 0; q < row; ++q)
                    {
                        const long m = q + 1 < R ? (long)(q + 1) * k * ts % N : 0;
                        const double ang = 2.0 * 3.141592653589793238462643383279502884 * (double)m / (double)N;
                        tw[o + (size_t)k * row + q] = make_float2((float)std::cos(ang), (float)(-std::sin(ang)));
                    }
            o += (size_t)ns * row;
            ns *= R;
        }
}

// One Stockham stage over an N-point LDS buffer of c2.
//   TWP: inter-stage twiddles as powers of one table root (1 VMEM load per
//        butterfly, R-2 extra complex multiplies); else R-1 table loads.
//   ORD: the last stage hands each lane its outputs in increasing index order (a
//        first-maximum scan needs it); without ORD it visits butterfly by
//        butterfly, so a partially filled pass is skipped as a whole instead of
//        predicating every output (order-free reductions: max, sum).
//   PADL (TWP_ >> 4): the buffer the last stage reads holds its N/RL-element
//        blocks at a stride of N/RL + PADL, so the penultimate stage's strided
//        writes spread over the LDS banks (bank model of MI355X_MICROARCH.md LDS:
//        PADL = 9 makes the 25 x 16 x 10 plan's transposes conflict-free).
template <int R, int NT, int N, int Ns, int TWP_, int TOFF, bool FIRST, bool LAST, bool PEN, bool ORD, class Load,
    class Store, class Hook>
__device__ __forceinline__ void stage(c2* lds, const float2* __restrict__ tw, Load& load, Store& store, Hook& hook)
{
    constexpr int TWP = TWP_ & 15;
    constexpr int PADL = (TWP_ >> 4) & 15;
    // LATE (TWP_ bit 8): the barrier that keeps the in-place Stockham exchange
    // safe (every wave's reads done before any wave's writes) moves from between
    // this stage's LDS reads and its butterflies to between the butterflies and its
    // writes, so the read latency overlaps the twiddles and the DFT; the last
    // stage needs none (its caller separates the next LDS writes with a barrier)
    constexpr bool LATE = ((TWP_ >> 8) & 1) != 0;
    constexpr bool DEFER = LATE && !FIRST && !LAST;
    // LASTNB (TWP_ bit 9): only the last stage's read barrier dropped -- it writes no
    // LDS, and every caller separates the next transform's LDS writes by a barrier of
    // its own (the correlate's row-statistic exchange, FourStepPkPlan's per-row sync)
    constexpr bool LASTNB = ((TWP_ >> 9) & 1) != 0;
    // elements before the TWP 3 table: N plus the last-stage pads (this stage is
    // the penultimate one whenever it reads the table)
    constexpr int DATA = N + (N / (Ns * R) - 1) * PADL;
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
                                v[b][r] = lds[jj + r * NB + (LAST ? r * PADL : 0)];
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
                                v[b][r] = lds[j + r * NB + (LAST ? r * PADL : 0)];
                        }
                }
        }
    if constexpr (FIRST)
        hook();
    else if constexpr (!LATE && !(LAST && LASTNB))
        __syncthreads();
    int kk[BPT];
#pragma unroll
    for (int b = 0; b < BPT; ++b)
        {
            const int j = (int)threadIdx.x + b * NT;
            kk[b] = 0;
            if (NB % NT == 0 || j < NB)
                {
                    int k = 0;
                    if constexpr (!FIRST)
                        {
                            k = j % Ns;
                            const int step = k * TSTRIDE;
                            // TWP 3: the middle stage reads its roots from the LDS copy
                            // of the per-stage table (PkPlan::run fills it), the last
                            // stage forms powers as TWP 1
                            constexpr int MODE = TWP == 3 ? (LAST ? 1 : 3) : TWP;
                            if constexpr (MODE == 3)
                                {
                                    const c2* lt = lds + DATA + k * lds_tw_row(R);
#pragma unroll
                                    for (int r = 1; r < R; ++r) v[b][r] = mul(v[b][r], lt[r - 1]);
                                }
                            else if constexpr (MODE == 2)
                                {
                                    // per-stage table (stage_tw_fill): row k holds W_N^{r k TSTRIDE},
                                    // r = 1..R-1, padded to an even count -> 16-byte loads
                                    constexpr int PR = stage_tw_row(R);
                                    const float4* t4 = reinterpret_cast<const float4*>(tw + TOFF + k * PR);
#pragma unroll
                                    for (int h = 0; h < PR / 2; ++h)
                                        {
                                            const float4 q = t4[h];
                                            const int r0 = 2 * h + 1;
                                            v[b][r0] = mul(v[b][r0], c2{q.x, q.y});
                                            if (r0 + 1 < R) v[b][r0 + 1] = mul(v[b][r0 + 1], c2{q.z, q.w});
                                        }
                                }
                            else if constexpr (MODE == 1)
                                {
                                    apply_powers<R>(v[b], from(tw[step]));
                                }
                            else
                                {
#pragma unroll
                                    for (int r = 1; r < R; ++r) v[b][r] = mul(v[b][r], from(tw[r * step]));
                                }
                        }
                    Dft<R>::run(v[b]);
                    kk[b] = k;
                    if constexpr (!LAST && !DEFER)
                        {
                            // block (j - k) R / (Ns R) = j / Ns of the last stage's input
                            const int base = (j - k) * R + k + (PEN ? (j / Ns) * PADL : 0);
#pragma unroll
                            for (int r = 0; r < R; ++r) lds[base + r * Ns] = v[b][r];
                        }
                }
        }
    if constexpr (DEFER)
        {
            __syncthreads();
#pragma unroll
            for (int b = 0; b < BPT; ++b)
                {
                    const int j = (int)threadIdx.x + b * NT;
                    if (NB % NT == 0 || j < NB)
                        {
                            const int k = kk[b];
                            const int base = (j - k) * R + k + (PEN ? (j / Ns) * PADL : 0);
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

// TOFF: the stage's first entry in the per-stage twiddle table (TWP == 2), which
// follows the N-entry W_N table; a stage of radix R over Ns-point sub-transforms
// holds Ns rows of stage_tw_row(R) entries.
template <int NT, int N, int Ns, int TWP, int TOFF, bool FIRST, bool ORD, int R, int... Rest, class Load, class Store,
    class Hook>
__device__ __forceinline__ void stages(c2* lds, const float2* __restrict__ tw, Load& load, Store& store, Hook& hook)
{
    constexpr bool LAST = sizeof...(Rest) == 0;
    constexpr bool PEN = sizeof...(Rest) == 1;
    stage<R, NT, N, Ns, TWP, TOFF, FIRST, LAST, PEN, ORD>(lds, tw, load, store, hook);
    constexpr int NEXT = FIRST ? TOFF : TOFF + Ns * stage_tw_row(R);
    if constexpr (!LAST) stages<NT, N, Ns * R, TWP, NEXT, false, ORD, Rest...>(lds, tw, load, store, hook);
}

// Compile-time packed plan.  load(b, r, i) -> c2 returns input element i
// (= j + r*N/R1 of this lane's b-th first-stage butterfly j); store(i, c2)
// consumes output element i, visited in increasing i per lane; hook() runs
// once the first stage's inputs are in registers (before its butterflies).
//   TWP: 0 inter-stage twiddles as R-1 loads from the W_N table, 1 as powers of one
//        loaded root, 2 from the per-stage table (stage_tw_fill: R-1 consecutive
//        roots per butterfly, 16-byte loads, no multiplies to form them).
template <int NT_, int TWP_, int... Rs>
struct PkPlan
{
    static constexpr int NT = NT_;
    static constexpr int TWP = TWP_ & 15;   // TWP_ >> 4: PADL (stage())
    static constexpr int PADL = (TWP_ >> 4) & 15;
    // entries of the twiddle table the kernels read: W_N (N) + the per-stage table
    static constexpr size_t tw_entries() { return (size_t)N + (TWP >= 2 ? stage_tw_entries<Rs...>() : 0); }
    // host: fill tw[N ..) with the per-stage table (tw[0, N) = W_N^m is the caller's)
    static void fill_stage_tw(float2* tw) { stage_tw_fill<Rs...>(tw, N); }
    static constexpr int N = (Rs * ...);
    static constexpr int nstages = sizeof...(Rs);
    static constexpr int R1 = fft::FirstRadix<Rs...>::value;
    static constexpr int BPT1 = fft::bpt_for(R1);
    static constexpr int NB1 = N / R1;
    static constexpr int R2 = fft::SecondRadix<Rs...>::value;
    static_assert(TWP != 3 || sizeof...(Rs) == 3, "TWP 3: one middle stage");
    // TWP 3: the middle stage's table (R1 rows of its R2 - 1 roots) after the data
    static constexpr int LTW = TWP == 3 ? R1 * lds_tw_row(R2) : 0;
    static constexpr int DATA = N + ((0, ..., Rs) - 1) * PADL;  // N + (RL - 1) PADL
    static constexpr size_t lds_bytes() { return (size_t)(DATA + LTW) * sizeof(c2); }
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
        if constexpr (TWP == 3)
            {
                // copy the middle stage's rows (global per-stage table at tw[N]) to
                // LDS; the first stage's barrier orders these writes before the
                // middle stage's reads, and a rewrite (next transform) stores the
                // same values
                constexpr int RW = stage_tw_row(R2);
                for (int i = (int)threadIdx.x; i < R1 * RW; i += NT)
                    {
                        const int row = i / RW, q = i - row * RW;
                        lds[DATA + row * lds_tw_row(R2) + q] = from(tw[N + i]);
                    }
            }
        stages<NT, N, 1, TWP_, N, true, ORD, Rs...>(lds, tw, load, store, hook);
    }
};


}  // namespace pk
}  // namespace gsdr
