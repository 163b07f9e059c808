// PCPS acquisition engine for MI355X (gfx950).
//
// Restates pcps_acquisition::acquisition_core
// (src/algorithms/acquisition/gnuradio_blocks/pcps_acquisition.cc:615-882) as a
// batched grid over (block, Doppler bin, PRN):
//
//   K_wipe    (init)  w_d[n] = exp(j*phi_n), phi accumulated in fp32 exactly like the
//                     generic volk_gnsssdr_s32f_sincos_32fc (pcps_acquisition.cc:233-246,298-305)
//   K_code    (init)  Cf_p = FFT(code_p placed in the FFT buffer)       (:176-209)
//   K_forward         X_{b,d} = FFT(x_b .* w_d)                          (:658-662)
//   K_correlate       per (b,d,p): |IFFT(X_{b,d} .* conj(Cf_p))|^2 in LDS, fused with the
//                     row reductions (max, first argmax, sum); the D x N magnitude grid
//                     of the reference never reaches HBM                  (:664-679)
//   K_reduce          per (b,p): grid maximum with the reference tie-break, CFAR input power,
//                     Gnss_Synchro fields                                (:511-543, :697-713)
//   K_second          per (b,p), peak-ratio mode only: recompute row d*, second peak outside
//                     the +-1 chip window with the reference's wrap      (:546-612)
#include "acq_impl.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <utility>
#include "gsdr_stream_internal.h"

namespace
{

// op: 0 run, 1 code fft, 2 dump spectra, 3 dump grid, 4 set attributes
int dispatch(gsdr_acq* a, int op, const void* iq, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* res, hipStream_t s, uint32_t aux)
{
    // the forward-spectrum layout of these launches: the main grid's (XMap), or the
    // plain one when a narrow step-two grid has replaced the wipe-off rows
    a->xm = (a->st2.active || a->d_wipe != a->d_wipe_grid) ? XMap{a->D, 0u, a->N} : a->xm_grid;
    if (a->variant >= 20) return gsdr_acq_impl::dispatch_four(a, op, iq, nblocks, stride, stamp0, res, s, aux);
    if (a->variant >= 10) return gsdr_acq_impl::dispatch_runtime(a, op, iq, nblocks, stride, stamp0, res, s, aux);
    return gsdr_acq_impl::dispatch_static(a, op, iq, nblocks, stride, stamp0, res, s, aux);
}

// Pick a compile-time plan when one matches N, else the smallest workgroup that
// admits a runtime plan.
constexpr size_t kLdsBytes = 160 * 1024;

bool choose_variant(gsdr_acq* a)
{
    const int N = (int)a->N;
    struct S
    {
        int id, n, nt;
        gsdr::fft::Plan p;
    };
    const S statics[] = {
        {1, StaticPlan<256, 20, 20, 10>::N, 256, StaticPlan<256, 20, 20, 10>::plan()},
        {2, StaticPlan<512, 20, 20, 20>::N, 512, StaticPlan<512, 20, 20, 20>::plan()},
        {3, StaticPlan<1024, 16, 10, 10, 10>::N, 1024, StaticPlan<1024, 16, 10, 10, 10>::plan()},
        {4, StaticPlan<256, 20, 10, 10>::N, 256, StaticPlan<256, 20, 10, 10>::plan()},
    };
    for (const S& st : statics)
        if (st.n == N)
            {
                a->variant = st.id;
                a->nt = st.nt;
                a->plan = st.p;
                return true;
            }
    const int ids[] = {10, 11, 12};
    const int nts[] = {256, 512, 1024};
    for (int i = 0; i < 3; ++i)
        if (gsdr::fft::make_plan(N, nts[i], a->plan) && a->plan.nstages >= 2 &&
            (size_t)N * sizeof(float2) + 16 * sizeof(RowStat) <= kLdsBytes)
            {
                a->variant = ids[i];
                a->nt = nts[i];
                return true;
            }
    // packed four-step (FourStepPkPlan) for the sizes of the GNSS configurations
    // beyond one workgroup's LDS: Galileo E1 4 / 8 ms at 8 Msps, 4 ms at 25 Msps,
    // 1 ms at 25 Msps (GSDR_ACQ_FOUR_GENERIC=1 keeps the generic four-step)
    {
        struct F
        {
            int id, n, r, n2;
        };
        const F fours[] = {{24, 32000, 8, 4000}, {25, 64000, 16, 4000}, {26, 100000, 25, 4000}, {27, 25000, 5, 5000}};
        const char* g = std::getenv("GSDR_ACQ_FOUR_GENERIC");
        for (const F& f : fours)
            if (f.n == N && !(g && std::atoi(g) != 0))
                {
                    a->variant = f.id;
                    a->nt = 256;
                    a->plan4 = gsdr::fft::Plan4{};
                    a->plan4.n = N;
                    a->plan4.r1 = f.r;
                    a->plan4.sub.n = f.n2;
                    a->plan4.sub.nstages = 0;  // compile-time sub-plan
                    a->plan.n = N;
                    return true;
                }
    }
    // four-step (fft_4step.h): N = R * N2, the largest register radix R whose N2
    // has an LDS plan
    const int radices[] = {25, 20, 16, 12, 10, 8};
    for (int R : radices)
        {
            if (N % R != 0) continue;
            const int N2 = N / R;
            if ((size_t)N2 * sizeof(float2) + 16 * sizeof(RowStat) > kLdsBytes) continue;
            for (int i = 0; i < 3; i += 2)  // 256 or 1024 threads (variants 20, 22)
                {
                    Plan sub{};
                    if (!gsdr::fft::make_plan(N2, nts[i], sub) || sub.nstages < 2) continue;
                    a->variant = 20 + i;
                    a->nt = nts[i];
                    a->plan4 = gsdr::fft::Plan4{};
                    a->plan4.n = N;
                    a->plan4.r1 = R;
                    a->plan4.sub = sub;
                    a->plan.n = N;  // buffer sizes
                    return true;
                }
        }
    return false;
}

}  // namespace

// ====================================================================== ABI
extern "C" {

int gsdr_acq_create(int device, const gsdr_acq_conf* conf, gsdr_acq** out)
{
    GSDR_REQUIRE(conf && out, GSDR_E_ARG, "gsdr_acq_create: null argument");
    *out = nullptr;
    GSDR_REQUIRE(conf->fs_in > 0 && conf->consumed_samples > 0, GSDR_E_ARG, "gsdr_acq_create: fs_in and consumed_samples must be > 0");
    GSDR_REQUIRE(conf->doppler_step > 0, GSDR_E_ARG, "gsdr_acq_create: doppler_step must be > 0");
    GSDR_REQUIRE(conf->item_type == GSDR_ITEM_GR_COMPLEX || conf->item_type == GSDR_ITEM_CSHORT ||
                     conf->item_type == GSDR_ITEM_IBYTE, GSDR_E_ARG,
        "gsdr_acq_create: unknown item type %d", conf->item_type);
    GSDR_REQUIRE(conf->max_prns > 0 && conf->max_blocks > 0, GSDR_E_ARG, "gsdr_acq_create: capacities must be > 0");
    GSDR_REQUIRE(conf->pfa >= 0.0f && conf->pfa <= 1.0f, GSDR_E_ARG, "gsdr_acq_create: pfa outside [0,1]");
    int ndev = 0;
    GSDR_HIP(hipGetDeviceCount(&ndev));
    GSDR_REQUIRE(device >= 0 && device < ndev, GSDR_E_ARG, "gsdr_acq_create: device %d of %d", device, ndev);
    gsdr::DeviceGuard g(device);

    gsdr_acq* a = new (std::nothrow) gsdr_acq();
    GSDR_REQUIRE(a, GSDR_E_ALLOC, "gsdr_acq_create: out of host memory");
    a->device = device;
    a->conf = *conf;
    if (a->conf.max_dwells == 0) a->conf.max_dwells = 1;
    // bit transition: every call decides on its own (the dwell counter is reset,
    // pcps_acquisition.cc:871-879) and the threshold uses one dwell (:908)
    if (a->conf.bit_transition_flag) a->conf.max_dwells = 1;
    a->K = a->conf.max_dwells;
    a->consumed = conf->consumed_samples;
    if (const char* w = std::getenv("GSDR_ACQ_WIPE"))
        {
            const std::string m(w);
            a->wipe_mode = m == "generic" ? GSDR_WIPE_GENERIC : (m == "avx2" ? GSDR_WIPE_AVX2 : GSDR_WIPE_EXACT);
        }
    // pcps_acquisition.cc:85-92
    uint32_t N = conf->fft_size;
    if (N == 0) N = (conf->sampled_ms == conf->ms_per_code || conf->sampled_ms == 0) ? a->consumed : 2 * a->consumed;
    if (N < a->consumed)
        {
            delete a;
            gsdr::set_error("gsdr_acq_create: fft_size %u < consumed_samples %u", N, a->consumed);
            return GSDR_E_ARG;
        }
    a->N = N;
    a->lead = N - a->consumed;
    a->eff = N;
    if (conf->bit_transition_flag)
        {
            if (N % 2 != 0)
                {
                    delete a;
                    gsdr::set_error("gsdr_acq_create: bit_transition_flag needs an even fft_size (%u)", N);
                    return GSDR_E_ARG;
                }
            a->lead = N / 2;
            a->eff = N / 2;
        }
    a->general = a->K > 1 || conf->bit_transition_flag;
    a->D = conf->num_doppler_bins;
    if (a->D == 0)
        a->D = (uint32_t)std::ceil((double)(conf->doppler_max - (-conf->doppler_max)) / (double)conf->doppler_step);
    if (a->D == 0)
        {
            delete a;
            gsdr::set_error("gsdr_acq_create: zero Doppler bins");
            return GSDR_E_ARG;
        }
    const bool ok = choose_variant(a);
    const bool four = a->variant >= 20;
    a->lds_bytes = (size_t)(four ? a->plan4.sub.n : N) * sizeof(float2) + 16 * sizeof(RowStat);
    if (!ok || a->lds_bytes > kLdsBytes)
        {
            delete a;
            gsdr::set_error("gsdr_acq_create: FFT size %u not supported (needs 2^a*3^b*5^c; up to 20352 points in "
                            "LDS, larger sizes as R*N2 with R in {8,10,12,16,20,25} and N2 <= 20352)", N);
            return GSDR_E_UNSUPPORTED;
        }
    int rc = dispatch(a, 4, nullptr, 0, 0, 0, nullptr, nullptr, 0);
    if (rc == GSDR_OK && four) rc = gsdr_acq_impl::setup_split(a);
    if (rc == GSDR_OK && !a->general && default_pk_variant(N) > 0)
        {
            int v = default_pk_variant(N);
            if (const char* e = std::getenv("GSDR_ACQ_CORR_VARIANT")) v = std::atoi(e);
            rc = gsdr_acq_impl::setup_corr_variant(a, v);
        }
    if (rc != GSDR_OK)
        {
            delete a;
            return rc;
        }
    const size_t nP = conf->max_prns, nB = conf->max_blocks;
    hipError_t e = hipStreamCreateWithFlags(&a->stream, hipStreamNonBlocking);

    const size_t tw_n = N;
    if (e == hipSuccess) e = hipMalloc(&a->d_tw, tw_n * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&a->d_wipe, (size_t)a->D * N * sizeof(float2));
    a->d_wipe_grid = a->d_wipe;
    if (e == hipSuccess) e = hipMalloc(&a->d_code_fft, nP * N * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&a->d_code_stage, nP * a->consumed * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&a->d_prn, nP * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&a->d_X, nB * a->K * a->D * N * sizeof(float2));
    if (e == hipSuccess) e = hipMalloc(&a->d_stats, nB * nP * a->K * a->D * sizeof(RowStat));
    if (e == hipSuccess) e = hipMalloc(&a->d_res, nB * nP * sizeof(gsdr_acq_result));
    if (e == hipSuccess) e = hipMalloc(&a->d_iq, nB * a->K * a->consumed * item_bytes(conf->item_type));
    if (a->general)
        {
            // accumulation rows held by running workgroups only: the chip's resident
            // workgroup count bounds the pool
            const int nslots = 256 * 32 / (a->nt / 64);
            a->acc_words = (nslots + 31) / 32;
            if (e == hipSuccess) e = hipMalloc(&a->d_resk, nB * nP * a->K * sizeof(gsdr_acq_result));
            if (e == hipSuccess) e = hipMalloc(&a->d_acc, (size_t)a->acc_words * 32 * a->eff * sizeof(float));
            if (e == hipSuccess) e = hipMalloc(&a->d_acc_slots, (size_t)a->acc_words * sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemset(a->d_acc_slots, 0, (size_t)a->acc_words * sizeof(uint32_t));
        }
    if (e == hipSuccess) e = hipMalloc(&a->d_grid, (size_t)a->D * N * sizeof(float));
    // split path with the peak-ratio statistic: one |R|^2 row per (block, PRN) for the
    // merged first/second-peak pass (acq_argmax_second_four_kernel)
    if (e == hipSuccess && a->split > 0 && !(conf->pfa > 0.0f))
        e = hipMalloc(&a->d_rowbuf, nB * nP * N * sizeof(float));
    // split path: the selected rows' first-maximum keys (acq_correlate_split_kernel<ARG>)
    if (e == hipSuccess && a->split > 0) e = hipMalloc(&a->d_keys, nB * nP * sizeof(unsigned long long));
    if (e == hipSuccess && a->split > 0) e = hipMalloc(&a->d_psum, nB * nP * 4 * sizeof(float));
    // split path: the two-launch forward's scratch rows (columns on every CU, then rows:
    // +8-12 % on C4 / C5 over one workgroup per spectrum, r04e)
    if (e == hipSuccess && a->split > 0) e = hipMalloc(&a->d_fscratch, nB * a->K * a->D * N * sizeof(float2));
    if (four)
        {
            // scratch slots: at least the resident workgroup count of the chip
            // (256 CUs x 32 waves / waves per workgroup), capped at 4 GiB
            int nslots = 256 * 32 / (a->nt / 64);
            while (nslots > 64 && (size_t)nslots * N * sizeof(float2) > (4ull << 30)) nslots /= 2;
            nslots = (nslots + 31) / 32 * 32;
            a->plan4.nwords = nslots / 32;
            if (e == hipSuccess) e = hipMalloc(&a->d_tw_sub, (size_t)a->plan4.sub.n * sizeof(float2));
            if (e == hipSuccess) e = hipMalloc(&a->d_scratch, (size_t)nslots * N * sizeof(float2));
            if (e == hipSuccess) e = hipMalloc(&a->d_slots, (size_t)a->plan4.nwords * sizeof(uint32_t));
            if (e == hipSuccess) e = hipMemset(a->d_slots, 0, (size_t)a->plan4.nwords * sizeof(uint32_t));
            if (e == hipSuccess)
                {
                    const int N2 = a->plan4.sub.n;
                    std::vector<float2> t2(N2);
                    for (int m = 0; m < N2; ++m)
                        {
                            const double ang = 2.0 * M_PI * (double)m / (double)N2;
                            t2[m] = make_float2((float)std::cos(ang), (float)(-std::sin(ang)));
                        }
                    e = hipMemcpy(a->d_tw_sub, t2.data(), N2 * sizeof(float2), hipMemcpyHostToDevice);
                }
            a->plan4.tw_sub = a->d_tw_sub;
            a->plan4.scratch = a->d_scratch;
            a->plan4.slots = a->d_slots;
        }
    if (e != hipSuccess)
        {
            gsdr::set_error("gsdr_acq_create: device allocation failed: %s", hipGetErrorString(e));
            gsdr_acq_destroy(a);
            return GSDR_E_ALLOC;
        }
    // twiddles W_N^m in double, rounded once
    std::vector<float2> tw(tw_n);
    for (uint32_t m = 0; m < N; ++m)
        {
            const double ang = 2.0 * M_PI * (double)m / (double)N;
            tw[m] = make_float2((float)std::cos(ang), (float)(-std::sin(ang)));
        }
    if ((e = hipMemcpy(a->d_tw, tw.data(), tw_n * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess)
        {
            gsdr::set_error("gsdr_acq_create: twiddle upload: %s", hipGetErrorString(e));
            gsdr_acq_destroy(a);
            return GSDR_E_DEVICE;
        }
    rc = rebuild_wipeoffs(a);
    if (rc != GSDR_OK)
        {
            gsdr_acq_destroy(a);
            return rc;
        }
    compute_threshold(a);
    *out = a;
    return GSDR_OK;
}

void gsdr_acq_destroy(gsdr_acq* a)
{
    if (!a) return;
    gsdr::DeviceGuard g(a->device);
    if (a->stream) (void)hipStreamSynchronize(a->stream);
    for (auto& r : a->prof_recs)
        {
            (void)hipEventDestroy(r.a);
            (void)hipEventDestroy(r.b);
        }
    for (hipEvent_t e : a->prof_pool) (void)hipEventDestroy(e);
    for (int i = 0; i < gsdr_acq::kSubs; ++i)
        {
            if (a->sub_done[i]) (void)hipEventDestroy(a->sub_done[i]);
            if (a->h_res[i]) (void)hipHostFree(a->h_res[i]);
        }
    void* bufs[] = {a->st2.d_wipe, a->st2.d_freq, a->d_tw, a->d_wipe, a->d_code_fft, a->d_code_stage, a->d_prn, a->d_X, a->d_stats, a->d_res,
        a->d_iq, a->d_grid, a->d_rowbuf, a->d_keys, a->d_psum, a->d_fscratch, a->d_dgrid, a->d_tw_sub, a->d_scratch, a->d_slots, a->d_resk, a->d_acc, a->d_acc_slots};
    for (void* p : bufs)
        if (p) (void)hipFree(p);
    if (a->stream) (void)hipStreamDestroy(a->stream);
    delete a;
}

int gsdr_acq_get_dims(const gsdr_acq* a, uint32_t* D, uint32_t* N)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_get_dims: null handle");
    if (D) *D = a->D;
    if (N) *N = a->N;
    return GSDR_OK;
}

int gsdr_acq_set_local_codes(gsdr_acq* a, const float* codes, const uint32_t* prn, uint32_t nprn)
{
    GSDR_REQUIRE(a && codes && prn, GSDR_E_ARG, "gsdr_acq_set_local_codes: null argument");
    GSDR_REQUIRE(nprn > 0 && nprn <= a->conf.max_prns, GSDR_E_ARG, "gsdr_acq_set_local_codes: nprn %u outside [1,%u]",
        nprn, a->conf.max_prns);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    GSDR_HIP(hipMemcpyAsync(a->d_code_stage, codes, (size_t)nprn * a->consumed * sizeof(float2),
        hipMemcpyHostToDevice, a->stream));
    GSDR_HIP(hipMemcpyAsync(a->d_prn, prn, nprn * sizeof(uint32_t), hipMemcpyHostToDevice, a->stream));
    int rc = dispatch(a, 1, nullptr, 0, 0, 0, nullptr, nullptr, nprn);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipStreamSynchronize(a->stream));
    a->nprn = nprn;
    return GSDR_OK;
}

int gsdr_acq_set_local_code(gsdr_acq* a, uint32_t slot, const float* code, uint32_t prn)
{
    GSDR_REQUIRE(a && code, GSDR_E_ARG, "gsdr_acq_set_local_code: null argument");
    GSDR_REQUIRE(slot < a->conf.max_prns && slot < 0xffffu, GSDR_E_ARG, "gsdr_acq_set_local_code: slot %u outside [0,%u)",
        slot, a->conf.max_prns);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    // ordered after every launch issued so far on the handle's stream (the slot's
    // previous spectrum may still be read by a submitted grid)
    GSDR_HIP(hipMemcpyAsync(a->d_code_stage + (size_t)slot * a->consumed, code, (size_t)a->consumed * sizeof(float2),
        hipMemcpyHostToDevice, a->stream));
    GSDR_HIP(hipMemcpyAsync(a->d_prn + slot, &prn, sizeof(uint32_t), hipMemcpyHostToDevice, a->stream));
    int rc = dispatch(a, 1, nullptr, 0, 0, 0, nullptr, nullptr, (slot << 16) | 1u);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipStreamSynchronize(a->stream));
    if (a->nprn <= slot) a->nprn = slot + 1;
    return GSDR_OK;
}

int gsdr_acq_set_active_prns(gsdr_acq* a, uint32_t nprn)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_active_prns: null handle");
    GSDR_REQUIRE(nprn > 0 && nprn <= a->conf.max_prns, GSDR_E_ARG, "gsdr_acq_set_active_prns: %u outside [1,%u]", nprn,
        a->conf.max_prns);
    std::lock_guard<std::mutex> lk(a->mu);
    a->nprn = nprn;
    return GSDR_OK;
}

int gsdr_acq_set_doppler(gsdr_acq* a, int32_t doppler_max, uint32_t doppler_step, int32_t doppler_center)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_doppler: null handle");
    GSDR_REQUIRE(doppler_step > 0, GSDR_E_ARG, "gsdr_acq_set_doppler: doppler_step must be > 0");
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    const uint32_t D = (uint32_t)std::ceil((double)(doppler_max - (-doppler_max)) / (double)doppler_step);
    GSDR_REQUIRE(a->conf.num_doppler_bins != 0 || D == a->D, GSDR_E_UNSUPPORTED,
        "gsdr_acq_set_doppler: changing the number of Doppler bins (%u -> %u) requires a new handle", a->D, D);
    a->conf.doppler_max = doppler_max;
    a->conf.doppler_step = doppler_step;
    a->conf.doppler_center = doppler_center;
    int rc = rebuild_wipeoffs(a);
    if (rc != GSDR_OK) return rc;
    compute_threshold(a);
    return GSDR_OK;
}

int gsdr_acq_set_wipeoff(gsdr_acq* a, int mode)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_wipeoff: null handle");
    GSDR_REQUIRE(mode == GSDR_WIPE_EXACT || mode == GSDR_WIPE_GENERIC || mode == GSDR_WIPE_AVX2, GSDR_E_ARG,
        "gsdr_acq_set_wipeoff: unknown mode %d", mode);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    a->wipe_mode = mode;
    return rebuild_wipeoffs(a);
}

int gsdr_acq_get_spectrum_reuse(const gsdr_acq* a, uint32_t* q, uint32_t* p)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_get_spectrum_reuse: null handle");
    if (q) *q = a->xm_grid.q;
    if (p) *p = a->xm_grid.p;
    return GSDR_OK;
}

int gsdr_acq_set_threshold(gsdr_acq* a, float threshold)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_threshold: null handle");
    a->threshold = threshold;
    return GSDR_OK;
}

int gsdr_acq_get_threshold(const gsdr_acq* a, float* threshold)
{
    GSDR_REQUIRE(a && threshold, GSDR_E_ARG, "gsdr_acq_get_threshold: null argument");
    *threshold = a->threshold;
    return GSDR_OK;
}

int gsdr_acq_run_device(gsdr_acq* a, const void* iq_dev, uint32_t nblocks, uint64_t stride, uint64_t stamp0,
    gsdr_acq_result* out_dev, void* stream)
{
    GSDR_REQUIRE(a && iq_dev && out_dev, GSDR_E_ARG, "gsdr_acq_run_device: null argument");
    GSDR_REQUIRE(a->nprn > 0, GSDR_E_STATE, "gsdr_acq_run_device: set_local_codes first");
    GSDR_REQUIRE(nblocks > 0 && nblocks <= a->conf.max_blocks, GSDR_E_ARG, "gsdr_acq_run_device: nblocks %u outside [1,%u]",
        nblocks, a->conf.max_blocks);
    GSDR_REQUIRE(stride >= a->consumed || nblocks == 1, GSDR_E_ARG, "gsdr_acq_run_device: block stride %llu < consumed %u",
        (unsigned long long)stride, a->consumed);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    hipStream_t s = stream ? (hipStream_t)stream : a->stream;
    return dispatch(a, 0, iq_dev, nblocks, stride, stamp0, out_dev, s, 0);
}

int gsdr_acq_run(gsdr_acq* a, const void* iq_host, uint32_t nblocks, uint64_t stamp0, gsdr_acq_result* out)
{
    GSDR_REQUIRE(a && iq_host && out, GSDR_E_ARG, "gsdr_acq_run: null argument");
    GSDR_REQUIRE(a->nprn > 0, GSDR_E_STATE, "gsdr_acq_run: set_local_codes first");
    GSDR_REQUIRE(nblocks > 0 && nblocks <= a->conf.max_blocks, GSDR_E_ARG, "gsdr_acq_run: nblocks %u outside [1,%u]",
        nblocks, a->conf.max_blocks);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    const size_t bytes = (size_t)nblocks * a->K * a->consumed * item_bytes(a->conf.item_type);
    GSDR_HIP(hipMemcpyAsync(a->d_iq, iq_host, bytes, hipMemcpyHostToDevice, a->stream));
    int rc = dispatch(a, 0, a->d_iq, nblocks, a->consumed, stamp0, a->d_res, a->stream, 0);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(out, a->d_res, (size_t)nblocks * a->nprn * sizeof(gsdr_acq_result), hipMemcpyDeviceToHost,
        a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_run_stream(gsdr_acq* a, gsdr_stream* ring, uint64_t first_sample, uint32_t nblocks, uint64_t stamp0,
    gsdr_acq_result* out)
{
    GSDR_REQUIRE(a && ring && out, GSDR_E_ARG, "gsdr_acq_run_stream: null argument");
    GSDR_REQUIRE(a->nprn > 0, GSDR_E_STATE, "gsdr_acq_run_stream: set_local_codes first");
    GSDR_REQUIRE(nblocks > 0 && nblocks <= a->conf.max_blocks, GSDR_E_ARG,
        "gsdr_acq_run_stream: nblocks %u outside [1,%u]", nblocks, a->conf.max_blocks);
    GSDR_REQUIRE(gsdr::stream_item_type(ring) == a->conf.item_type, GSDR_E_ARG,
        "gsdr_acq_run_stream: ring item type %d != acquisition item type %d", gsdr::stream_item_type(ring),
        a->conf.item_type);
    GSDR_REQUIRE(gsdr::stream_device(ring) == a->device, GSDR_E_ARG,
        "gsdr_acq_run_stream: ring on device %d, acquisition handle on device %d", gsdr::stream_device(ring), a->device);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    {
        gsdr::StreamReader rd(ring);  // ring lock from view to reader-event record
        const void* iq = nullptr;
        int rc = rd.view(first_sample, (uint64_t)nblocks * a->K * a->consumed, &iq);
        if (rc != GSDR_OK) return rc;
        rc = rd.acquire(a->stream);
        if (rc != GSDR_OK) return rc;
        rc = dispatch(a, 0, iq, nblocks, a->consumed, stamp0, a->d_res, a->stream, 0);
        if (rc != GSDR_OK) return rc;
        rc = rd.release(a->stream);
        if (rc != GSDR_OK) return rc;
    }
    GSDR_HIP(hipMemcpyAsync(out, a->d_res, (size_t)nblocks * a->nprn * sizeof(gsdr_acq_result), hipMemcpyDeviceToHost,
        a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_submit_stream(gsdr_acq* a, gsdr_stream* ring, uint64_t first_sample, uint32_t nblocks, uint64_t stamp0)
{
    GSDR_REQUIRE(a && ring, GSDR_E_ARG, "gsdr_acq_submit_stream: null argument");
    GSDR_REQUIRE(a->nprn > 0, GSDR_E_STATE, "gsdr_acq_submit_stream: set_local_codes first");
    GSDR_REQUIRE(nblocks > 0 && nblocks <= a->conf.max_blocks, GSDR_E_ARG,
        "gsdr_acq_submit_stream: nblocks %u outside [1,%u]", nblocks, a->conf.max_blocks);
    GSDR_REQUIRE(gsdr::stream_item_type(ring) == a->conf.item_type, GSDR_E_ARG,
        "gsdr_acq_submit_stream: ring item type %d != acquisition item type %d", gsdr::stream_item_type(ring),
        a->conf.item_type);
    GSDR_REQUIRE(gsdr::stream_device(ring) == a->device, GSDR_E_ARG,
        "gsdr_acq_submit_stream: ring on device %d, acquisition handle on device %d", gsdr::stream_device(ring), a->device);
    std::lock_guard<std::mutex> lk(a->mu);
    GSDR_REQUIRE(a->sub_count < gsdr_acq::kSubs, GSDR_E_STATE,
        "gsdr_acq_submit_stream: %d submissions in flight, collect the oldest first", gsdr_acq::kSubs);
    gsdr::DeviceGuard g(a->device);
    const int slot = (a->sub_head + a->sub_count) % gsdr_acq::kSubs;
    if (!a->h_res[slot])
        {
            GSDR_HIP(hipHostMalloc(&a->h_res[slot],
                (size_t)a->conf.max_blocks * a->conf.max_prns * sizeof(gsdr_acq_result), hipHostMallocDefault));
            GSDR_HIP(hipEventCreateWithFlags(&a->sub_done[slot], hipEventDisableTiming));
        }
    {
        gsdr::StreamReader rd(ring);  // ring lock from view to reader-event record
        const void* iq = nullptr;
        int rc = rd.view(first_sample, (uint64_t)nblocks * a->K * a->consumed, &iq);
        if (rc != GSDR_OK) return rc;
        rc = rd.acquire(a->stream);
        if (rc != GSDR_OK) return rc;
        rc = dispatch(a, 0, iq, nblocks, a->consumed, stamp0, a->d_res, a->stream, 0);
        if (rc != GSDR_OK) return rc;
        rc = rd.release(a->stream);
        if (rc != GSDR_OK) return rc;
    }
    GSDR_HIP(hipMemcpyAsync(a->h_res[slot], a->d_res, (size_t)nblocks * a->nprn * sizeof(gsdr_acq_result),
        hipMemcpyDeviceToHost, a->stream));
    GSDR_HIP(hipEventRecord(a->sub_done[slot], a->stream));
    a->sub_blocks[slot] = nblocks;
    a->sub_nprn[slot] = a->nprn;
    a->sub_count++;
    return GSDR_OK;
}

int gsdr_acq_collect(gsdr_acq* a, gsdr_acq_result* out, uint32_t* nblocks, uint32_t* nprn)
{
    GSDR_REQUIRE(a && out, GSDR_E_ARG, "gsdr_acq_collect: null argument");
    std::lock_guard<std::mutex> lk(a->mu);
    GSDR_REQUIRE(a->sub_count > 0, GSDR_E_STATE, "gsdr_acq_collect: nothing submitted");
    gsdr::DeviceGuard g(a->device);
    const int slot = a->sub_head;
    a->sub_head = (a->sub_head + 1) % gsdr_acq::kSubs;
    a->sub_count--;
    GSDR_HIP(hipEventSynchronize(a->sub_done[slot]));
    std::memcpy(out, a->h_res[slot], (size_t)a->sub_blocks[slot] * a->sub_nprn[slot] * sizeof(gsdr_acq_result));
    if (nblocks) *nblocks = a->sub_blocks[slot];
    if (nprn) *nprn = a->sub_nprn[slot];
    return GSDR_OK;
}

int gsdr_acq_run_dwell(gsdr_acq* a, const void* iq_host, uint32_t dwell, uint64_t stamp, gsdr_acq_result* out)
{
    GSDR_REQUIRE(a && iq_host && out, GSDR_E_ARG, "gsdr_acq_run_dwell: null argument");
    GSDR_REQUIRE(a->nprn > 0, GSDR_E_STATE, "gsdr_acq_run_dwell: set_local_codes first");
    GSDR_REQUIRE(dwell < a->conf.max_dwells, GSDR_E_ARG, "gsdr_acq_run_dwell: dwell %u outside [0,%u)", dwell,
        a->conf.max_dwells);
    GSDR_REQUIRE(!a->st2.active, GSDR_E_STATE, "gsdr_acq_run_dwell: step two in progress");
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    if (!a->d_dgrid)
        GSDR_HIP(hipMalloc(&a->d_dgrid, (size_t)a->conf.max_prns * a->D * a->eff * sizeof(float)));
    GSDR_HIP(hipMemcpyAsync(a->d_iq, iq_host, (size_t)a->consumed * item_bytes(a->conf.item_type),
        hipMemcpyHostToDevice, a->stream));
    int rc = dispatch(a, 5, nullptr, 1, a->consumed, stamp, a->d_res, a->stream, dwell);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(out, a->d_res, (size_t)a->nprn * sizeof(gsdr_acq_result), hipMemcpyDeviceToHost,
        a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_dump_spectra(gsdr_acq* a, const void* iq_host, float* spectra_host)
{
    GSDR_REQUIRE(a && iq_host && spectra_host, GSDR_E_ARG, "gsdr_acq_dump_spectra: null argument");
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    GSDR_HIP(hipMemcpyAsync(a->d_iq, iq_host, (size_t)a->consumed * item_bytes(a->conf.item_type),
        hipMemcpyHostToDevice, a->stream));
    int rc = dispatch(a, 2, nullptr, 1, 0, 0, nullptr, a->stream, 0);
    if (rc != GSDR_OK) return rc;
    // row d of block 0 wherever the layout keeps it (XMap: a window of a shared spectrum)
    for (uint32_t d = 0; d < a->D; ++d)
        GSDR_HIP(hipMemcpyAsync(spectra_host + (size_t)d * a->N * 2, a->d_X + a->xm.off(0, d),
            (size_t)a->N * sizeof(float2), hipMemcpyDeviceToHost, a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_dump_grid(gsdr_acq* a, const void* iq_host, uint32_t prn_slot, float* grid_host)
{
    GSDR_REQUIRE(a && iq_host && grid_host, GSDR_E_ARG, "gsdr_acq_dump_grid: null argument");
    GSDR_REQUIRE(prn_slot < a->nprn, GSDR_E_ARG, "gsdr_acq_dump_grid: prn_slot %u >= nprn %u", prn_slot, a->nprn);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    GSDR_HIP(hipMemcpyAsync(a->d_iq, iq_host, (size_t)a->consumed * item_bytes(a->conf.item_type),
        hipMemcpyHostToDevice, a->stream));
    int rc = dispatch(a, 3, nullptr, 1, 0, 0, nullptr, a->stream, prn_slot);
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(grid_host, a->d_grid, (size_t)a->D * a->N * sizeof(float), hipMemcpyDeviceToHost,
        a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_dump_grid_step_two(gsdr_acq* a, const void* iq_host, uint32_t prn_slot, float doppler_center_hz,
    float* grid_host)
{
    GSDR_REQUIRE(a && iq_host && grid_host, GSDR_E_ARG, "gsdr_acq_dump_grid_step_two: null argument");
    GSDR_REQUIRE(prn_slot < a->nprn, GSDR_E_ARG, "gsdr_acq_dump_grid_step_two: prn_slot %u >= nprn %u", prn_slot,
        a->nprn);
    GSDR_REQUIRE(a->st2.nbins > 0, GSDR_E_STATE, "gsdr_acq_dump_grid_step_two: gsdr_acq_set_step_two first");
    GSDR_REQUIRE(a->st2.nbins <= a->D, GSDR_E_UNSUPPORTED,
        "gsdr_acq_dump_grid_step_two: %u narrow bins exceed the grid buffer's %u rows", a->st2.nbins, a->D);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    const uint32_t nb = a->st2.nbins;
    // update_grid_doppler_wipeoffs_step2 (pcps_acquisition.cc:307-314), as gsdr_acq_run_step_two
    const float half = (float)std::floor((double)nb / 2.0);
    std::vector<float> freqs(nb);
    for (uint32_t d = 0; d < nb; ++d)
        {
            volatile float dop = ((float)d - half) * a->st2.step;
            freqs[d] = doppler_center_hz + dop;
        }
    GSDR_HIP(hipMemcpyAsync(a->d_iq, iq_host, (size_t)a->consumed * item_bytes(a->conf.item_type),
        hipMemcpyHostToDevice, a->stream));
    GSDR_HIP(hipMemcpyAsync(a->st2.d_freq, freqs.data(), nb * sizeof(float), hipMemcpyHostToDevice, a->stream));
    hipLaunchKernelGGL(acq_wipeoff_kernel, dim3(nb), dim3(256), 0, a->stream, a->st2.d_wipe, a->N,
        (float)a->conf.fs_in, 0, 0, 0, 0, (const float*)a->st2.d_freq, a->wipe_mode);
    GSDR_HIP(hipGetLastError());
    // the grid dump on a one-PRN view with the narrow Doppler rows
    const uint32_t D0 = a->D, P0 = a->nprn;
    float2* const wipe0 = a->d_wipe;
    float2* const code0 = a->d_code_fft;
    a->D = nb;
    a->nprn = 1;
    a->d_wipe = a->st2.d_wipe;
    a->d_code_fft = code0 + (size_t)prn_slot * a->N;
    const int rc = dispatch(a, 3, nullptr, 1, 0, 0, nullptr, a->stream, 0);
    a->D = D0;
    a->nprn = P0;
    a->d_wipe = wipe0;
    a->d_code_fft = code0;
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(grid_host, a->d_grid, (size_t)nb * a->N * sizeof(float), hipMemcpyDeviceToHost,
        a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_set_step_two(gsdr_acq* a, uint32_t num_doppler_bins_step2, float doppler_step2, float pfa2)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_step_two: null handle");
    GSDR_REQUIRE(num_doppler_bins_step2 > 0, GSDR_E_ARG, "gsdr_acq_set_step_two: zero bins");
    GSDR_REQUIRE(num_doppler_bins_step2 <= a->D * a->conf.max_blocks, GSDR_E_UNSUPPORTED,
        "gsdr_acq_set_step_two: %u bins exceed the handle's spectrum capacity (%u bins x %u blocks)",
        num_doppler_bins_step2, a->D, a->conf.max_blocks);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    GSDR_HIP(hipStreamSynchronize(a->stream));
    if (a->st2.d_wipe) (void)hipFree(a->st2.d_wipe);
    if (a->st2.d_freq) (void)hipFree(a->st2.d_freq);
    a->st2.d_wipe = nullptr;
    a->st2.d_freq = nullptr;
    const size_t rows = (size_t)a->conf.max_prns * num_doppler_bins_step2;
    GSDR_HIP(hipMalloc(&a->st2.d_wipe, rows * a->N * sizeof(float2)));
    GSDR_HIP(hipMalloc(&a->st2.d_freq, rows * sizeof(float)));
    a->st2.nbins = num_doppler_bins_step2;
    a->st2.step = doppler_step2;
    // Acq_Conf: pfa_second_step outside (0, 1] falls back to pfa (acq_conf.cc:72-76)
    a->st2.pfa2 = (pfa2 <= 0.0f || pfa2 > 1.0f) ? a->conf.pfa : pfa2;
    return GSDR_OK;
}

int gsdr_acq_get_step_two_threshold(const gsdr_acq* a, float* threshold)
{
    GSDR_REQUIRE(a && threshold, GSDR_E_ARG, "gsdr_acq_get_step_two_threshold: null argument");
    GSDR_REQUIRE(a->st2.nbins > 0, GSDR_E_STATE, "gsdr_acq_get_step_two_threshold: gsdr_acq_set_step_two first");
    *threshold = step_two_threshold(a);
    return GSDR_OK;
}

int gsdr_acq_run_step_two(gsdr_acq* a, const void* iq_host, uint32_t nsel, const uint32_t* prn_slots,
    const float* doppler_center_hz, const float* coarse_input_power, uint64_t stamp, gsdr_acq_result* out)
{
    GSDR_REQUIRE(a && iq_host && prn_slots && doppler_center_hz && coarse_input_power && out, GSDR_E_ARG,
        "gsdr_acq_run_step_two: null argument");
    GSDR_REQUIRE(a->st2.nbins > 0, GSDR_E_STATE, "gsdr_acq_run_step_two: gsdr_acq_set_step_two first");
    GSDR_REQUIRE(nsel > 0 && nsel <= a->nprn, GSDR_E_ARG, "gsdr_acq_run_step_two: %u PRNs outside [1,%u]", nsel,
        a->nprn);
    for (uint32_t i = 0; i < nsel; ++i)
        GSDR_REQUIRE(prn_slots[i] < a->nprn, GSDR_E_ARG, "gsdr_acq_run_step_two: slot %u >= nprn %u", prn_slots[i],
            a->nprn);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    const uint32_t nb = a->st2.nbins;
    // update_grid_doppler_wipeoffs_step2 (pcps_acquisition.cc:307-314), float arithmetic
    const float half = (float)std::floor((double)nb / 2.0);
    std::vector<float> freqs((size_t)nsel * nb);
    for (uint32_t i = 0; i < nsel; ++i)
        for (uint32_t d = 0; d < nb; ++d)
            {
                volatile float dop = ((float)d - half) * a->st2.step;
                freqs[(size_t)i * nb + d] = doppler_center_hz[i] + dop;
            }
    GSDR_HIP(hipMemcpyAsync(a->d_iq, iq_host, (size_t)a->K * a->consumed * item_bytes(a->conf.item_type),
        hipMemcpyHostToDevice, a->stream));
    GSDR_HIP(hipMemcpyAsync(a->st2.d_freq, freqs.data(), freqs.size() * sizeof(float), hipMemcpyHostToDevice,
        a->stream));
    hipLaunchKernelGGL(acq_wipeoff_kernel, dim3(nsel * nb), dim3(256), 0, a->stream, a->st2.d_wipe, a->N,
        (float)a->conf.fs_in, 0, 0, 0, 0, (const float*)a->st2.d_freq, a->wipe_mode);
    GSDR_HIP(hipGetLastError());
    // one narrow grid per PRN (each has its own centre): the engine's launches on a
    // one-PRN view of the handle
    const uint32_t D0 = a->D, P0 = a->nprn;
    float2* const wipe0 = a->d_wipe;
    float2* const code0 = a->d_code_fft;
    uint32_t* const prn0 = a->d_prn;
    const float thr = step_two_threshold(a);
    int rc = GSDR_OK;
    for (uint32_t i = 0; i < nsel && rc == GSDR_OK; ++i)
        {
            a->D = nb;
            a->nprn = 1;
            a->d_wipe = a->st2.d_wipe + (size_t)i * nb * a->N;
            a->d_code_fft = code0 + (size_t)prn_slots[i] * a->N;
            a->d_prn = prn0 + prn_slots[i];
            a->st2.active = true;
            a->st2.center = doppler_center_hz[i];
            a->st2.ip = coarse_input_power[i];
            a->st2.threshold = thr;
            rc = dispatch(a, 0, a->d_iq, 1, a->consumed, stamp, a->d_res + i, a->stream, 0);
        }
    a->D = D0;
    a->nprn = P0;
    a->d_wipe = wipe0;
    a->d_code_fft = code0;
    a->d_prn = prn0;
    a->st2.active = false;
    if (rc != GSDR_OK) return rc;
    GSDR_HIP(hipMemcpyAsync(out, a->d_res, (size_t)nsel * sizeof(gsdr_acq_result), hipMemcpyDeviceToHost, a->stream));
    GSDR_HIP(hipStreamSynchronize(a->stream));
    return GSDR_OK;
}

int gsdr_acq_set_cu_mask(gsdr_acq* a, const uint32_t* mask, int n_words)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_cu_mask: null handle");
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    return gsdr::replace_stream(&a->stream, mask, n_words);
}

int gsdr_acq_set_profiling(gsdr_acq* a, int enable)
{
    GSDR_REQUIRE(a, GSDR_E_ARG, "gsdr_acq_set_profiling: null handle");
    std::lock_guard<std::mutex> lk(a->mu);
    a->profiling = enable != 0;
    if (a->profiling)
        {
            // pre-create the stage events, so a profiled run records pooled events
            // instead of calling hipEventCreate inside the caller's timed loop (8 per
            // call: four stages bracketed; read_profile returns them to the pool)
            gsdr::DeviceGuard g(a->device);
            while (a->prof_pool.size() + 2 * a->prof_recs.size() < 1024)
                {
                    hipEvent_t e = nullptr;
                    if (hipEventCreate(&e) != hipSuccess) break;
                    a->prof_pool.push_back(e);
                }
        }
    return GSDR_OK;
}

int gsdr_acq_read_profile_ex(gsdr_acq* a, double* stage_ms, uint32_t* launches, double* stage_busy_ms)
{
    GSDR_REQUIRE(a && stage_ms && launches, GSDR_E_ARG, "gsdr_acq_read_profile: null argument");
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    for (int i = 0; i < 4; ++i)
        {
            stage_ms[i] = 0.0;
            launches[i] = 0;
            if (stage_busy_ms) stage_busy_ms[i] = 0.0;
        }
    // per launch: duration, and [start, end) against the first record's start event
    std::vector<std::pair<double, double>> iv[4];
    hipEvent_t ref = a->prof_recs.empty() ? nullptr : a->prof_recs.front().a;
    for (auto& r : a->prof_recs)
        {
            GSDR_HIP(hipEventSynchronize(r.b));
            float ms = 0.0f, t0 = 0.0f, t1 = 0.0f;
            GSDR_HIP(hipEventElapsedTime(&ms, r.a, r.b));
            GSDR_HIP(hipEventElapsedTime(&t0, ref, r.a));
            GSDR_HIP(hipEventElapsedTime(&t1, ref, r.b));
            stage_ms[r.stage] += ms;
            launches[r.stage] += 1;
            iv[r.stage].emplace_back(t0, t1);
        }
    // busy time of a stage: the union of its launch intervals (launches of one stage
    // overlap when runs of the handle are issued on several streams)
    if (stage_busy_ms)
        for (int i = 0; i < 4; ++i)
            {
                std::sort(iv[i].begin(), iv[i].end());
                double busy = 0.0, lo = 0.0, hi = -1e300;
                for (const auto& x : iv[i])
                    {
                        if (x.first > hi)
                            {
                                if (hi > lo) busy += hi - lo;
                                lo = x.first;
                                hi = x.second;
                            }
                        else if (x.second > hi)
                            hi = x.second;
                    }
                if (hi > lo) busy += hi - lo;
                stage_busy_ms[i] = busy;
            }
    for (auto& r : a->prof_recs)
        {
            a->prof_pool.push_back(r.a);
            a->prof_pool.push_back(r.b);
        }
    a->prof_recs.clear();
    return GSDR_OK;
}

int gsdr_acq_read_profile_intervals(gsdr_acq* a, const void* ref_event, int stage, double* start_ms, double* end_ms,
    uint32_t max_n, uint32_t* n)
{
    GSDR_REQUIRE(a && ref_event && n && (max_n == 0 || (start_ms && end_ms)), GSDR_E_ARG,
        "gsdr_acq_read_profile_intervals: null argument");
    GSDR_REQUIRE(stage >= 0 && stage < 4, GSDR_E_ARG, "gsdr_acq_read_profile_intervals: stage %d", stage);
    std::lock_guard<std::mutex> lk(a->mu);
    gsdr::DeviceGuard g(a->device);
    hipEvent_t ref = (hipEvent_t)const_cast<void*>(ref_event);
    uint32_t k = 0;
    for (auto& r : a->prof_recs)
        {
            if (r.stage != stage) continue;
            if (k < max_n)
                {
                    GSDR_HIP(hipEventSynchronize(r.b));
                    float t0 = 0.0f, t1 = 0.0f;
                    GSDR_HIP(hipEventElapsedTime(&t0, ref, r.a));
                    GSDR_HIP(hipEventElapsedTime(&t1, ref, r.b));
                    start_ms[k] = t0;
                    end_ms[k] = t1;
                }
            ++k;
        }
    *n = k;
    return GSDR_OK;
}

int gsdr_acq_read_profile(gsdr_acq* a, double* stage_ms, uint32_t* launches)
{
    return gsdr_acq_read_profile_ex(a, stage_ms, launches, nullptr);
}

}  // extern "C"
