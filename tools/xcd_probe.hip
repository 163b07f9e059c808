// Which XCD runs workgroup id? Reads HW_REG_XCC_ID (s_getreg, gfx94x/gfx950) in every
// workgroup of a 1-D grid shaped like the C2 correlate launch (256 lanes, ~32 KB LDS)
// and reports how often xcc == id % 8, plus the first ids' placement.  Also with two
// such grids in flight on two streams (the bench's two acquisition chains).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned* out, int spin)
{
    extern __shared__ float lds[];
    if (threadIdx.x == 0)
        {
            const unsigned x = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((4 - 1) << 11));
            out[blockIdx.x] = x & 15u;
        }
    // a little work so workgroups overlap like the real kernel's
    float a = threadIdx.x;
    for (int i = 0; i < spin; ++i) a = a * 1.0000001f + 0.5f;
    lds[threadIdx.x] = a;
    __syncthreads();
    if (lds[(threadIdx.x + 1) & 255] == -1.0f) out[0] = 99;
}

static void report(const char* tag, const std::vector<unsigned>& h)
{
    size_t same = 0, rot = 0, n = h.size();
    const unsigned off = h[0] & 7u;
    std::vector<size_t> cnt(16, 0);
    for (size_t i = 0; i < n; ++i)
        {
            same += (h[i] == (i & 7u));
            rot += (h[i] == ((i + off) & 7u));
            cnt[h[i] & 15u]++;
        }
    printf("%s: n=%zu xcc==id%%8 for %.3f, xcc==(id+%u)%%8 for %.3f; per-xcc", tag, n, (double)same / n, off,
        (double)rot / n);
    for (int x = 0; x < 8; ++x) printf(" %zu", cnt[x]);
    printf("; first 24:");
    for (int i = 0; i < 24; ++i) printf(" %u", h[i]);
    printf("\n");
}

int main()
{
    const int n = 32 * 81 * 32;  // one correlate launch of 32 blocks
    unsigned *d1, *d2;
    (void)hipMalloc(&d1, n * sizeof(unsigned));
    (void)hipMalloc(&d2, n * sizeof(unsigned));
    hipStream_t s1, s2;
    hipStreamCreate(&s1);
    hipStreamCreate(&s2);
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 32768);
    std::vector<unsigned> h(n);
    for (int spin : {0, 2000, 40000})
        {
            hipLaunchKernelGGL(probe, dim3(n), dim3(256), 32768, s1, d1, spin);
            hipStreamSynchronize(s1);
            hipMemcpy(h.data(), d1, n * sizeof(unsigned), hipMemcpyDeviceToHost);
            char tag[64];
            snprintf(tag, sizeof tag, "single spin=%d", spin);
            report(tag, h);
            hipLaunchKernelGGL(probe, dim3(n), dim3(256), 32768, s1, d1, spin);
            hipLaunchKernelGGL(probe, dim3(n), dim3(256), 32768, s2, d2, spin);
            hipDeviceSynchronize();
            hipMemcpy(h.data(), d1, n * sizeof(unsigned), hipMemcpyDeviceToHost);
            snprintf(tag, sizeof tag, "two streams A spin=%d", spin);
            report(tag, h);
            hipMemcpy(h.data(), d2, n * sizeof(unsigned), hipMemcpyDeviceToHost);
            snprintf(tag, sizeof tag, "two streams B spin=%d", spin);
            report(tag, h);
        }
    return 0;
}
