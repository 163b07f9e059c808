// Error reporting, device queries and the threshold's special function.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdarg>
#include <cstdio>

#include "gsdr_internal.h"

namespace
{
thread_local char g_last_error[512] = "";
}

namespace gsdr
{

void set_error(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

// Q(a, x) = 1 - P(a, x) = exp(-x) * sum_{k<a} x^k / k!  for integer a >= 1.
static long double upper_reg_gamma_int(int a, long double x)
{
    long double term = 1.0L, sum = 1.0L;
    for (int k = 1; k < a; ++k)
        {
            term *= x / (long double)k;
            sum += term;
        }
    return std::exp(-x) * sum;
}

// Inverse of the regularised lower incomplete gamma function for integer shape:
// the role Boost's gamma_p_inv plays in pcps_acquisition::calculate_threshold
// (pcps_acquisition.cc:908), where the shape is 2*max_dwells.  Solves
// Q(a, x) = 1 - p by bracketing + Newton on log Q (Q is tiny for the p ~ 1 - 1e-8
// of acquisition thresholds, so work with the upper tail directly).
double gamma_p_inv_int(int a, double p)
{
    if (a < 1 || !(p > 0.0)) return 0.0;
    if (p >= 1.0) return INFINITY;
    const long double q = 1.0L - (long double)p;
    const long double lq = std::log(q);
    long double lo = 0.0L, hi = 1.0L;
    while (std::log(upper_reg_gamma_int(a, hi)) > lq) hi *= 2.0L;
    long double x = 0.5L * (lo + hi);
    for (int it = 0; it < 200; ++it)
        {
            const long double Q = upper_reg_gamma_int(a, x);
            const long double f = std::log(Q) - lq;  // decreasing in x
            if (f > 0)
                lo = x;
            else
                hi = x;
            // d log Q / dx = -x^(a-1) e^-x / ((a-1)! Q)
            long double lg = (a - 1) * std::log(x) - x - std::lgamma((long double)a);
            long double deriv = -std::exp(lg) / Q;
            long double xn = x - f / deriv;
            if (!(xn > lo && xn < hi)) xn = 0.5L * (lo + hi);
            if (std::fabs(xn - x) <= 1e-17L * std::fabs(x)) return (double)xn;
            x = xn;
        }
    return (double)x;
}

int replace_stream(hipStream_t* stream, const uint32_t* mask, int n_words)
{
    GSDR_REQUIRE(n_words >= 0 && (n_words == 0 || mask), GSDR_E_ARG, "cu mask: bad argument");
    hipStream_t s = nullptr;
    if (n_words == 0)
        {
            GSDR_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
        }
    else
        {
            bool any = false;
            for (int i = 0; i < n_words; ++i) any |= mask[i] != 0u;
            GSDR_REQUIRE(any, GSDR_E_ARG, "cu mask: no CU selected");
            GSDR_HIP(hipExtStreamCreateWithCUMask(&s, (uint32_t)n_words, mask));
        }
    if (*stream)
        {
            (void)hipStreamSynchronize(*stream);
            (void)hipStreamDestroy(*stream);
        }
    *stream = s;
    return GSDR_OK;
}

}  // namespace gsdr

extern "C" {

const char* gsdr_last_error(void) { return g_last_error; }

int gsdr_abi_version(void) { return GSDR_ABI_VERSION; }

int gsdr_device_count(int* count)
{
    GSDR_REQUIRE(count, GSDR_E_ARG, "gsdr_device_count: null argument");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e == hipErrorNoDevice)
        {
            *count = 0;
            return GSDR_OK;
        }
    GSDR_HIP(e);
    *count = n;
    return GSDR_OK;
}

int gsdr_host_register(void* ptr, size_t bytes)
{
    GSDR_REQUIRE(ptr && bytes > 0, GSDR_E_ARG, "gsdr_host_register: null or empty buffer");
    GSDR_HIP(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
    return GSDR_OK;
}

int gsdr_host_unregister(void* ptr)
{
    GSDR_REQUIRE(ptr, GSDR_E_ARG, "gsdr_host_unregister: null buffer");
    GSDR_HIP(hipHostUnregister(ptr));
    return GSDR_OK;
}

}  // extern "C"
