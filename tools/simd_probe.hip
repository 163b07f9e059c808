// Which SIMD runs wave w of a workgroup?  Reads HW_REG_HW_ID (s_getreg; SIMD_ID bits
// 5:4, CU_ID 11:8) in every wave of a 1-D grid shaped like the C2 correlate launch
// (256 lanes = 4 waves, ~32 KB LDS, 4 workgroups per CU) and reports, per wave index,
// the SIMD histogram and how often SIMD == (w + s) % 4 for a per-workgroup start s.
// If wave w always lands on SIMD w, a stage that leaves wave 3 idle idles SIMD 3.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(256) probe(unsigned* out, int spin)
{
    extern __shared__ float lds[];
    const unsigned hw = __builtin_amdgcn_s_getreg(4 | (0 << 6) | ((32 - 1) << 11));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = hw;
    float a = threadIdx.x;
    for (int i = 0; i < spin; ++i) a = a * 1.0000001f + 0.5f;
    lds[threadIdx.x] = a;
    __syncthreads();
    if (lds[(threadIdx.x + 1) & 255] == -1.0f) out[0] = 99;
}

int main()
{
    const int n = 32 * 81 * 32;
    unsigned* d;
    (void)hipMalloc(&d, n * 4 * sizeof(unsigned));
    (void)hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 32768);
    std::vector<unsigned> h(n * 4);
    for (int spin : {0, 4000})
        {
            hipLaunchKernelGGL(probe, dim3(n), dim3(256), 32768, 0, d, spin);
            (void)hipDeviceSynchronize();
            (void)hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
            size_t hist[4][4] = {}, consistent = 0, ident = 0;
            for (int b = 0; b < n; ++b)
                {
                    const unsigned s0 = (h[b * 4] >> 4) & 3u;
                    bool cons = true;
                    for (int w = 0; w < 4; ++w)
                        {
                            const unsigned sm = (h[b * 4 + w] >> 4) & 3u;
                            hist[w][sm]++;
                            cons = cons && sm == ((s0 + w) & 3u);
                        }
                    consistent += cons;
                    ident += (s0 == 0 && cons);
                }
            printf("spin=%d: workgroups %d, SIMD == (start + w) %% 4 in %.3f, start 0 in %.3f\n", spin, n,
                (double)consistent / n, (double)ident / n);
            for (int w = 0; w < 4; ++w)
                printf("  wave %d: SIMD histogram %zu %zu %zu %zu\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
            printf("  first 8 workgroups (simd of waves 0..3, cu):");
            for (int b = 0; b < 8; ++b)
                printf(" [%u%u%u%u cu%u]", (h[b * 4] >> 4) & 3u, (h[b * 4 + 1] >> 4) & 3u, (h[b * 4 + 2] >> 4) & 3u,
                    (h[b * 4 + 3] >> 4) & 3u, (h[b * 4] >> 8) & 15u);
            printf("\n");
        }
    return 0;
}
