// rocFFT A/B for the large-N acquisition grids (north_star names
// rocFFT for the acquisition transforms, the reference's are FFTW plans,
// src/algorithms/libs/gnss_sdr_fft.h:27-60).  A measuring tool, not product code:
// the library path materialises the grid the split kernels never write --
//   product   Y[d][p] = conj(X_d) . C_p             (D x P rows of N complex, HBM)
//   rocFFT    batched in-place forward transforms  (|IFFT(Y)| = |FFT(conj Y)|,
//             the conjugation folded into the product)
//   rowmax    max |Y|^2 per row                    (the split kernels' STAT 2)
// and times each with HIP events on one stream, per block of the grid, beside the
// library's bare transform rate.  One JSON line per N.
//   rocfft_ab [reps]
#include <hip/hip_runtime.h>
#include <rocfft/rocfft.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK_HIP(x)                                                                                  \
    do                                                                                                \
        {                                                                                             \
            hipError_t e_ = (x);                                                                      \
            if (e_ != hipSuccess)                                                                     \
                {                                                                                     \
                    std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
                    std::exit(1);                                                                     \
                }                                                                                     \
        }                                                                                             \
    while (0)
#define CHECK_FFT(x)                                                                  \
    do                                                                                \
        {                                                                             \
            rocfft_status s_ = (x);                                                   \
            if (s_ != rocfft_status_success)                                          \
                {                                                                     \
                    std::fprintf(stderr, "%s:%d %s: rocfft status %d\n", __FILE__, __LINE__, #x, (int)s_); \
                    std::exit(1);                                                     \
                }                                                                     \
        }                                                                             \
    while (0)

// Y[(d P + p) N + k] = conj(conj(X_d[k]) C_p[k]) = X_d[k] conj(C_p[k]): the forward
// transform of conj(Y) has |.| = |IFFT(Y)| N, as the engine's correlate
__global__ void product_kernel(const float2* __restrict__ X, const float2* __restrict__ C, float2* __restrict__ Y,
    int N, int P, size_t total)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x)
        {
            const size_t row = i / N, k = i - row * N;
            const size_t d = row / P, p = row - d * P;
            const float2 x = X[d * N + k], c = C[p * N + k];
            Y[i] = make_float2(x.x * c.x + x.y * c.y, x.y * c.x - x.x * c.y);
        }
}

// one 256-lane workgroup per row: max |Y|^2
__global__ void __launch_bounds__(256) rowmax_kernel(const float2* __restrict__ Y, float* __restrict__ out, int N)
{
    const float2* y = Y + (size_t)blockIdx.x * N;
    float m = 0.0f;
    for (int k = threadIdx.x; k < N; k += 256)
        {
            const float2 v = y[k];
            m = fmaxf(m, v.x * v.x + v.y * v.y);
        }
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    __shared__ float red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

int main(int argc, char** argv)
{
    const int reps = argc > 1 ? std::atoi(argv[1]) : 5;
    CHECK_FFT(rocfft_setup());
    struct Cfg
    {
        const char* name;
        int N, P, D;
    };
    // the shipped grids (profiles/configs_bench.py): C5 GPS / BeiDou, C4 4 ms, C4 bit
    // transition (the library computes all 64000 outputs), C5 Galileo
    const Cfg cfgs[] = {{"C5 GPS/BDS 32 PRN x 81 Doppler", 25000, 32, 81},
        {"C4 Galileo 4 ms 36 PRN x 81 Doppler", 32000, 36, 81},
        {"C4 Galileo bit transition 36 PRN x 81 Doppler", 64000, 36, 81},
        {"C5 Galileo 4 ms 36 PRN x 41 Doppler", 100000, 36, 41}};
    hipStream_t st;
    CHECK_HIP(hipStreamCreate(&st));
    for (const Cfg& c : cfgs)
        {
            const size_t N = (size_t)c.N, rows = (size_t)c.D * c.P, total = rows * N;
            std::vector<float2> h((size_t)(c.D + c.P) * N);
            srand(1);
            for (auto& v : h) v = make_float2((float)(rand() & 0xffff) / 65536.0f - 0.5f, (float)(rand() & 0xffff) / 65536.0f - 0.5f);
            float2 *X, *C, *Y;
            float* rmax;
            CHECK_HIP(hipMalloc(&X, (size_t)c.D * N * sizeof(float2)));
            CHECK_HIP(hipMalloc(&C, (size_t)c.P * N * sizeof(float2)));
            CHECK_HIP(hipMalloc(&Y, total * sizeof(float2)));
            CHECK_HIP(hipMalloc(&rmax, rows * sizeof(float)));
            CHECK_HIP(hipMemcpy(X, h.data(), (size_t)c.D * N * sizeof(float2), hipMemcpyHostToDevice));
            CHECK_HIP(hipMemcpy(C, h.data() + (size_t)c.D * N, (size_t)c.P * N * sizeof(float2), hipMemcpyHostToDevice));
            rocfft_plan plan = nullptr;
            const size_t len = N;
            CHECK_FFT(rocfft_plan_create(&plan, rocfft_placement_inplace, rocfft_transform_type_complex_forward,
                rocfft_precision_single, 1, &len, rows, nullptr));
            size_t wbytes = 0;
            CHECK_FFT(rocfft_plan_get_work_buffer_size(plan, &wbytes));
            void* work = nullptr;
            rocfft_execution_info info = nullptr;
            CHECK_FFT(rocfft_execution_info_create(&info));
            CHECK_FFT(rocfft_execution_info_set_stream(info, st));
            if (wbytes)
                {
                    CHECK_HIP(hipMalloc(&work, wbytes));
                    CHECK_FFT(rocfft_execution_info_set_work_buffer(info, work, wbytes));
                }
            hipEvent_t e0, e1, e2, e3;
            CHECK_HIP(hipEventCreate(&e0));
            CHECK_HIP(hipEventCreate(&e1));
            CHECK_HIP(hipEventCreate(&e2));
            CHECK_HIP(hipEventCreate(&e3));
            void* bufs[1] = {Y};
            double t_prod = 0, t_fft = 0, t_max = 0;
            for (int r = 0; r < reps + 1; ++r)
                {
                    CHECK_HIP(hipEventRecord(e0, st));
                    hipLaunchKernelGGL(product_kernel, dim3(4096), dim3(256), 0, st, X, C, Y, c.N, c.P, total);
                    CHECK_HIP(hipEventRecord(e1, st));
                    CHECK_FFT(rocfft_execute(plan, bufs, nullptr, info));
                    CHECK_HIP(hipEventRecord(e2, st));
                    hipLaunchKernelGGL(rowmax_kernel, dim3((unsigned)rows), dim3(256), 0, st, Y, rmax, c.N);
                    CHECK_HIP(hipEventRecord(e3, st));
                    CHECK_HIP(hipEventSynchronize(e3));
                    float a, b, d;
                    CHECK_HIP(hipEventElapsedTime(&a, e0, e1));
                    CHECK_HIP(hipEventElapsedTime(&b, e1, e2));
                    CHECK_HIP(hipEventElapsedTime(&d, e2, e3));
                    if (r > 0)
                        {
                            t_prod += a / reps;
                            t_fft += b / reps;
                            t_max += d / reps;
                        }
                }
            // per block: the P x D correlate transforms of one N-sample block
            const double t_block = (t_prod + t_fft + t_max) * 1e-3;
            const double flops = (double)rows * (5.0 * N * std::log2((double)N) + 11.0 * N);
            const double fft_flops = (double)rows * 5.0 * N * std::log2((double)N);
            std::printf("{\"tool\": \"rocfft_ab\", \"grid\": \"%s\", \"N\": %zu, \"P\": %d, \"D\": %d, \"rocfft_work_bytes\": %zu, "
                        "\"ms_product\": %.4f, \"ms_rocfft\": %.4f, \"ms_rowmax\": %.4f, \"ms_per_block\": %.4f, "
                        "\"correlate_msps\": %.3f, \"correlate_tflops\": %.2f, \"rocfft_alone_tflops\": %.2f, "
                        "\"grid_bytes\": %zu}\n",
                c.name, N, c.P, c.D, wbytes, t_prod, t_fft, t_max, t_block * 1e3, N / t_block / 1e6,
                flops / t_block / 1e12, fft_flops / (t_fft * 1e-3) / 1e12, total * sizeof(float2));
            std::fflush(stdout);
            CHECK_FFT(rocfft_execution_info_destroy(info));
            CHECK_FFT(rocfft_plan_destroy(plan));
            if (work) CHECK_HIP(hipFree(work));
            CHECK_HIP(hipFree(X));
            CHECK_HIP(hipFree(C));
            CHECK_HIP(hipFree(Y));
            CHECK_HIP(hipFree(rmax));
        }
    CHECK_FFT(rocfft_cleanup());
    return 0;
}
