// Probe: which hardware CUs (XCC, SE, CU) run the workgroups of a stream
// created with hipExtStreamCreateWithCUMask, for a few masks.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>
__global__ void who(unsigned* out)
{
    if (threadIdx.x == 0)
        {
            unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));      // HW_REG_HW_ID (gfx9: id 4)
            unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));    // HW_REG_XCC_ID (gfx940+: id 20)
            out[2 * blockIdx.x] = hw;
            out[2 * blockIdx.x + 1] = xcc;
            for (volatile int i = 0; i < 2000; ++i) {}
        }
}
int main()
{
    const int nblk = 4096;
    unsigned* d;
    hipMalloc(&d, nblk * 2 * sizeof(unsigned));
    std::vector<unsigned> h(nblk * 2);
    std::vector<std::vector<uint32_t>> masks;
    masks.push_back(std::vector<uint32_t>(8, 0xffffffffu));
    { std::vector<uint32_t> m(8, 0); m[0] = 0xffu; masks.push_back(m); }                 // bits 0..7
    { std::vector<uint32_t> m(8, 0); for (int x = 0; x < 8; ++x) m[x] = 1u; masks.push_back(m); }  // bit 32x
    { std::vector<uint32_t> m(8, 0); m[0] = 0x1u; masks.push_back(m); }                  // bit 0
    { std::vector<uint32_t> m(8, 0xffffffffu); for (int x = 0; x < 8; ++x) m[x] &= ~1u; masks.push_back(m); }
    for (size_t mi = 0; mi < masks.size(); ++mi)
        {
            hipStream_t s;
            hipError_t e = hipExtStreamCreateWithCUMask(&s, 256, masks[mi].data());
            if (e != hipSuccess) { printf("mask %zu: create failed %s\n", mi, hipGetErrorString(e)); continue; }
            hipLaunchKernelGGL(who, dim3(nblk), dim3(64), 0, s, d);
            hipStreamSynchronize(s);
            hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
            std::set<std::tuple<unsigned, unsigned, unsigned>> cus;
            for (int b = 0; b < nblk; ++b)
                {
                    unsigned hw = h[2 * b], xcc = h[2 * b + 1] & 0xf;
                    unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 0x7;
                    cus.insert({xcc, se * 2 + sh, cu});
                }
            printf("mask %zu: %zu distinct CUs;", mi, cus.size());
            int k = 0;
            for (auto& t : cus) { if (k++ < 12) printf(" (x%u,s%u,c%u)", std::get<0>(t), std::get<1>(t), std::get<2>(t)); }
            printf("\n");
            hipStreamDestroy(s);
        }
    return 0;
}
