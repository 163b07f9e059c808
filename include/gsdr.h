/*
 * gsdr.h — C ABI of the MI355X-native GNSS acquisition + tracking correlator engine.
 *
 * This is the drop-in boundary for GNSS-SDR's two data-parallel hot paths:
 *
 *  - PCPS acquisition: replaces the compute of pcps_acquisition
 *    (src/algorithms/acquisition/gnuradio_blocks/pcps_acquisition.cc:176-209
 *    set_local_code, :233-305 Doppler grid, :511-612 statistics, :615-882
 *    acquisition_core, :894-909 calculate_threshold), batched over PRNs and over
 *    consecutive input blocks.
 *
 *  - Tracking multicorrelator: replaces Cpu_Multicorrelator_Real_Codes
 *    (src/algorithms/tracking/libs/cpu_multicorrelator_real_codes.h:37-61, .cc:36-167)
 *    and Cpu_Multicorrelator (src/algorithms/tracking/libs/cpu_multicorrelator.h:37-58),
 *    i.e. the VOLK-GNSSSDR resampler + rotator-dot-product pair, fused into one
 *    HIP launch batched over channels.
 *
 * Conventions
 *  - Every function returns int: GSDR_OK (0) or a negative GSDR_E* code.  The
 *    thread-local message of the last failure is gsdr_last_error().  No C++
 *    exception crosses this boundary.
 *  - Plain pointers and sizes only.  "host" pointers are ordinary CPU memory;
 *    "dev" pointers are HIP device memory on the handle's device; "stream" is a
 *    hipStream_t passed as void* (NULL = the handle's own stream).
 *  - Complex samples are interleaved float pairs (gr_complex / std::complex<float>),
 *    cshort samples are interleaved int16 pairs (lv_16sc_t).
 *  - A handle is owned by one caller at a time; distinct handles may be used
 *    concurrently from different threads (GNU Radio thread-per-block model).
 */
#ifndef GSDR_H
#define GSDR_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GSDR_ABI_VERSION 1

#define GSDR_OK 0
#define GSDR_E_ARG (-1)         /* invalid argument (≙ std::invalid_argument in Acq_Conf) */
#define GSDR_E_DEVICE (-2)      /* HIP runtime / device error */
#define GSDR_E_ALLOC (-3)       /* device or host allocation failed */
#define GSDR_E_STATE (-4)       /* call not valid in the handle's current state */
#define GSDR_E_UNSUPPORTED (-5) /* configuration outside what the engine implements */

/* Sample item types (Acq_Conf::item_type, acq_conf.h:42; item_type_size). */
#define GSDR_ITEM_GR_COMPLEX 0 /* complex<float>, 8 bytes */
#define GSDR_ITEM_CSHORT 1     /* complex<int16>, 4 bytes (also ishort: Ishort_To_Complex reads the same pairs) */
/* interleaved int8 I,Q, 2 bytes: SignalSource.item_type=byte through Ibyte_To_Complex
 * (data_type_adapter/adapters/ibyte_to_complex.cc:39, gr::blocks::interleaved_char_to_complex
 * with scale 1): converted exactly to complex<float> inside the kernels' loads. */
#define GSDR_ITEM_IBYTE 2

/* Float association used for the resampler code-phase index:
 * GSDR_ASSOC_GENERIC: floor((step*n + shift) - rem)   KERN/32f_xn_resampler_32f_xn.h:73
 * GSDR_ASSOC_AVX:     floor(step*n + (shift - rem))   KERN/32f_xn_resampler_32f_xn.h:384-390
 * The x86 VOLK dispatcher selects the AVX protokernel, so that is the default. */
#define GSDR_ASSOC_GENERIC 0
#define GSDR_ASSOC_AVX 1

const char* gsdr_last_error(void);
int gsdr_abi_version(void);
/* Number of HIP devices visible to this process. */
int gsdr_device_count(int* count);
/* Page-lock a host buffer (the flowgraph's sample buffer upstream of the blocks) so
 * gsdr_stream_push / the host-input calls copy it to HBM by DMA without a staging
 * copy; gsdr_host_unregister before the buffer is freed.  No reference counterpart
 * (GNU Radio buffers are pageable; gr-cuda style custom buffers would pin them). */
int gsdr_host_register(void* ptr, size_t bytes);
int gsdr_host_unregister(void* ptr);

/* ======================================================================== */
/* Device IQ ring indexed by absolute sample count                           */
/* ======================================================================== */
/*
 * The input stream uploaded once per GPU and read in place by every consumer --
 * the acquisition grid and the tracking channel pool -- by absolute sample
 * index: the nitems_read index dll_pll_veml_tracking consumes by
 * (dll_pll_veml_tracking.cc:1797,1818,2122) and the sample counter
 * pcps_acquisition stamps its results with (pcps_acquisition.cc:968,1009).  In a
 * GNU Radio flowgraph one block pushes each general_work call's items; the
 * acquisition and tracking blocks then launch on windows of the ring instead of
 * copying their own host buffers.
 *
 * capacity_items ring positions (sample % capacity) plus a mirror of the first
 * max_window_items positions, so every window of up to max_window_items items
 * is one contiguous device span.  The ring keeps the last capacity_items items.
 */
typedef struct gsdr_stream gsdr_stream;

int gsdr_stream_create(int device, int item_type, uint64_t capacity_items, uint64_t max_window_items, gsdr_stream** out);
void gsdr_stream_destroy(gsdr_stream* stream);
/* Append n items (item_type of the ring) whose first one is absolute input sample
 * first_sample; pushes are contiguous (first_sample = the previous push's end;
 * the first push sets the origin).  Asynchronous H2D on the ring's copy stream,
 * ordered after every consumer launch issued so far (no overwrite of data in
 * use); n <= capacity_items.
 * Lifetime of iq_host: the copy reads it after the call returns (from page-locked
 * memory, gsdr_host_register, it is a DMA straight from the caller's buffer), so
 * the n items must stay valid and unchanged until the push has landed:
 * gsdr_stream_landed reports *landed >= first_sample + n, or
 * gsdr_stream_wait_landed(stream, first_sample + n) returned.  A GNU Radio block
 * that pushes its input items therefore consumes (consume_each) only items that
 * landed -- the scheduler recycles consumed items upstream
 * (dll_pll_veml_tracking.cc:2119). */
int gsdr_stream_push(gsdr_stream* stream, const void* iq_host, uint64_t first_sample, uint64_t n);
/* Every item before *landed is in device memory: the host memory of the pushes that
 * ended there may be reused.  Non-blocking. */
int gsdr_stream_landed(gsdr_stream* stream, uint64_t* landed);
/* Waits until every push holding an item before `upto` has landed. */
int gsdr_stream_wait_landed(gsdr_stream* stream, uint64_t upto);
/* The longest contiguous window ending at the newest item: [*first_sample,
 * *first_sample + *n_items). */
int gsdr_stream_span(gsdr_stream* stream, uint64_t* first_sample, uint64_t* n_items);
/* Device pointer of items [first_sample, first_sample + n_items) after the pushes
 * so far have landed (synchronises with the copy stream); GSDR_E_ARG if the window
 * is not (or no longer) in the ring.  For host-synchronous readers: the pointer
 * stays valid until the next push.  A reader whose kernels run on a stream uses
 * the pair below instead. */
int gsdr_stream_window(gsdr_stream* stream, uint64_t first_sample, uint64_t n_items, const void** iq_dev);
/* Asynchronous reader: the same window, with consumer_stream (a hipStream_t)
 * made to wait for the pushes so far; after enqueuing its reads the caller calls
 * gsdr_stream_release(stream, consumer_stream), and every later push waits for
 * those reads before it overwrites ring positions.  Between the two calls the
 * window is open: a push from another thread that would overwrite it blocks
 * until the release, and such a push from the thread that opened it returns
 * GSDR_E_STATE (release first).  With pushes from another thread, the caller keeps
 * the two calls and its launches between them free of any wait on that thread.
 * The library's own consumers (gsdr_acq_run_stream, gsdr_trk_run_stream) hold the
 * ring lock from window to release. */
int gsdr_stream_window_async(gsdr_stream* stream, uint64_t first_sample, uint64_t n_items, void* consumer_stream,
    const void** iq_dev);
int gsdr_stream_release(gsdr_stream* stream, void* consumer_stream);
/* The device the ring lives on (a consumer handle must be on the same device). */
int gsdr_stream_device(const gsdr_stream* stream, int* device);

/* ======================================================================== */
/* Acquisition — PCPS (pcps_acquisition)                                     */
/* ======================================================================== */

typedef struct gsdr_acq gsdr_acq;

/* Mirrors the Acq_Conf fields (acq_conf.h:33-82) that drive acquisition_core. */
typedef struct gsdr_acq_conf
{
    int64_t fs_in;                /* sampling rate after optional resampling [sps]   (resampled_fs) */
    uint32_t consumed_samples;    /* samples per block = sampled_ms*samples_per_ms    (pcps_acquisition.cc:71) */
    uint32_t fft_size;            /* 0 -> derived as in pcps_acquisition.cc:85-92 */
    float samples_per_code;       /* Acq_Conf::samples_per_code */
    uint32_t samples_per_chip;    /* Acq_Conf::samples_per_chip (peak-ratio exclusion window) */
    int32_t doppler_max;          /* [Hz] */
    uint32_t doppler_step;        /* [Hz] */
    int32_t doppler_center;       /* [Hz] */
    int32_t doppler_bias;         /* [Hz] FDMA bias (is_fdma, pcps_acquisition.cc:212-230) */
    uint32_t num_doppler_bins;    /* 0 -> ceil(2*doppler_max/doppler_step)            (pcps_acquisition.cc:264) */
    float pfa;                    /* > 0: CFAR max/input-power statistic; == 0: first/second peak */
    uint32_t max_dwells;          /* non-coherent dwells per acquisition attempt (forced to 1 with bit_transition_flag) */
    int32_t bit_transition_flag;  /* consumed = 2 x sampled span, code in the second half, outputs [N/2, N) */
    int32_t item_type;            /* GSDR_ITEM_* */
    uint32_t max_prns;            /* capacity: PRNs per batch */
    uint32_t max_blocks;          /* capacity: blocks per call */
    uint32_t sampled_ms;          /* Acq_Conf::sampled_ms */
    uint32_t ms_per_code;         /* Acq_Conf::ms_per_code */
} gsdr_acq_conf;

/* One acquisition outcome per (block, PRN): the Gnss_Synchro fields written by
 * acquisition_core (pcps_acquisition.cc:697-713) plus the statistic inputs. */
typedef struct gsdr_acq_result
{
    uint32_t prn;
    uint32_t doppler_index;   /* d* */
    uint32_t code_phase;      /* indext: n* in the (effective) FFT row */
    int32_t doppler_hz;       /* Acq_doppler_hz */
    float peak;               /* grid maximum |R|^2 */
    float input_power;        /* CFAR: mean |R|^2 of row (d*+D/2)%D / 2 / dwells; 0 for peak-ratio */
    float second_peak;        /* peak-ratio: second peak outside +-1 chip; 0 for CFAR */
    float test_statistic;     /* d_test_statistics */
    double acq_delay_samples; /* Acq_delay_samples = fmod(indext, samples_per_code) */
    uint64_t samplestamp;     /* Acq_samplestamp_samples */
    int32_t positive;         /* test_statistic > threshold */
    int32_t num_dwells;       /* dwells integrated when the decision was taken (1..max_dwells) */
} gsdr_acq_result;

int gsdr_acq_create(int device, const gsdr_acq_conf* conf, gsdr_acq** out);
void gsdr_acq_destroy(gsdr_acq* acq);

/* Doppler bins D actually used, and the FFT size. */
int gsdr_acq_get_dims(const gsdr_acq* acq, uint32_t* num_doppler_bins, uint32_t* fft_size);

/* set_local_code for a batch of PRNs (pcps_acquisition.cc:176-209): codes is
 * nprn rows of consumed_samples complex<float> (host); the engine places each in
 * the FFT buffer, transforms and conjugates on the device.  prn[] are the PRN ids
 * reported back in gsdr_acq_result. */
int gsdr_acq_set_local_codes(gsdr_acq* acq, const float* codes, const uint32_t* prn, uint32_t nprn);
/* set_local_code of one PRN slot (pcps_acquisition.cc:176-209, called once per PRN
 * assignment by the channel, gps_l1_ca_pcps_acquisition.cc:151-170): code is
 * consumed_samples complex<float> (host), transformed into slot `slot` of the
 * handle's code spectra; the other slots keep theirs.  Extends the active PRN
 * count to slot + 1 if needed.  Ordered after the launches already issued. */
int gsdr_acq_set_local_code(gsdr_acq* acq, uint32_t slot, const float* code, uint32_t prn);
/* Number of PRN slots [0, nprn) the grid launches search (each with a spectrum set
 * by gsdr_acq_set_local_code[s]). */
int gsdr_acq_set_active_prns(gsdr_acq* acq, uint32_t nprn);

/* Doppler setters (AcquisitionInterface, acquisition_interface.h:56-59).  They
 * rebuild the Doppler wipe-off grid on the device. */
int gsdr_acq_set_doppler(gsdr_acq* acq, int32_t doppler_max, uint32_t doppler_step, int32_t doppler_center);

/* Carrier wipe-off model of the Doppler grid (update_local_carrier,
 * pcps_acquisition.cc:233-246, through volk_gnsssdr_s32f_sincos_32fc):
 *   GSDR_WIPE_EXACT   exp(-j 2 pi f n / fs), phase reduced and evaluated in fp64,
 *                     rounded once (default);
 *   GSDR_WIPE_GENERIC the generic protokernel bit for bit (KERN/s32f_sincos_32fc.h:390-403:
 *                     one fp32 phase accumulator, cosf / sinf);
 *   GSDR_WIPE_AVX2    the a_avx2 protokernel the reference dispatches on AVX2 x86-64
 *                     (:448-627: eight fp32 accumulators, Cephes polynomials).
 * The protokernels' fp32 phase accumulators drift from the exact carrier (GPS 4 Msps:
 * 1e-3 / 2e-5 rad over 1 ms; Galileo 8 Msps, 8 ms: 0.15 / 0.01 rad); DESIGN.md 3.
 * With EXACT and Doppler bins commensurate with the FFT bins (doppler_step * N / fs =
 * p / q, q <= D / 2) the forward pass computes q spectra per block and every Doppler
 * row is an exact circular shift of one of them (gsdr_acq_get_spectrum_reuse).
 * Initial mode: GSDR_ACQ_WIPE=exact|generic|avx2 in the environment, else EXACT. */
#define GSDR_WIPE_EXACT 0
#define GSDR_WIPE_GENERIC 1
#define GSDR_WIPE_AVX2 2
int gsdr_acq_set_wipeoff(gsdr_acq* acq, int mode);
/* The forward-spectrum reuse in effect: *q spectra per block (== D: none), each
 * Doppler class step shifting by *p bins. */
int gsdr_acq_get_spectrum_reuse(const gsdr_acq* acq, uint32_t* q, uint32_t* p);

/* Threshold: set explicitly (set_threshold) or computed from pfa exactly as
 * calculate_threshold (pcps_acquisition.cc:894-909). */
int gsdr_acq_set_threshold(gsdr_acq* acq, float threshold);
int gsdr_acq_get_threshold(const gsdr_acq* acq, float* threshold);

/* Synchronous drop-in: nblocks acquisition attempts over consecutive blocks of
 * consumed_samples items (item_type) from host memory.  Attempt i integrates up
 * to max_dwells blocks (block j = i*max_dwells + k for dwell k, sample stamp
 * stamp0 + j*consumed) and reports, per PRN, the first dwell whose statistic
 * crosses the threshold or else the last (acquisition_core's dwell loop,
 * pcps_acquisition.cc:781-869); with max_dwells = 1 an attempt is one block.
 * out: nblocks*nprn results, attempt-major (host). */
int gsdr_acq_run(gsdr_acq* acq, const void* iq_host, uint32_t nblocks, uint64_t stamp0, gsdr_acq_result* out);

/* acquisition_core's dwell loop one block per call, as the reference block runs
 * it (pcps_acquisition.cc:637-680, :781-829): dwell = the call's
 * d_num_noncoherent_integrations_counter - 1 (0 <= dwell < max_dwells).  Dwell 0
 * starts a device-resident |R|^2 grid per PRN, later dwells add this block's
 * |R|^2 into it (volk_32f_x2_add_32f); the statistic is evaluated on the
 * accumulated grid with the counter as the CFAR divisor (:534), against the
 * max_dwells threshold (:908).  iq_host: one block (consumed_samples items);
 * out: nprn results (num_dwells = dwell + 1).  Synchronous.  The caller keeps
 * the dwell FSM (positive / next dwell / negative after max_dwells). */
int gsdr_acq_run_dwell(gsdr_acq* acq, const void* iq_host, uint32_t dwell, uint64_t stamp, gsdr_acq_result* out);

/* Device-resident form: iq_dev holds nblocks*max_dwells blocks, block j starting
 * at item j*block_stride_items.  Results are written to out_dev (device memory,
 * nblocks*nprn).  Asynchronous on stream; no host synchronisation. */
int gsdr_acq_run_device(gsdr_acq* acq, const void* iq_dev, uint32_t nblocks, uint64_t block_stride_items,
    uint64_t stamp0, gsdr_acq_result* out_dev, void* stream);

/* Ring form: nblocks attempts on the ring's items from absolute sample
 * first_sample on (the nblocks*max_dwells consecutive blocks gsdr_acq_run would
 * read from a contiguous host buffer), results to out_host (nblocks*nprn), sample
 * stamps from stamp0 as in gsdr_acq_run.  The launch waits for the ring's
 * pushes on the device (no host synchronisation before it) and is ordered before
 * later pushes overwrite the window.  Synchronous (results on the host). */
int gsdr_acq_run_stream(gsdr_acq* acq, gsdr_stream* stream, uint64_t first_sample, uint32_t nblocks, uint64_t stamp0,
    gsdr_acq_result* out_host);
/* Asynchronous ring form (the batched acquisition service's call, gnss_flowgraph.cc:
 * 1796-1901 answered per block): the grids of nblocks attempts from first_sample are
 * launched on the handle's stream with the results copied into the handle's pinned
 * buffer; returns without waiting.  gsdr_acq_collect waits for them and copies the
 * nblocks * nprn results (block-major, nprn = the active count at submission) to
 * out_host.  Up to two submissions in flight per handle (the second queued behind
 * the first on the handle's stream), collected oldest first. */
int gsdr_acq_submit_stream(gsdr_acq* acq, gsdr_stream* stream, uint64_t first_sample, uint32_t nblocks,
    uint64_t stamp0);
int gsdr_acq_collect(gsdr_acq* acq, gsdr_acq_result* out_host, uint32_t* nblocks, uint32_t* nprn);

/* The reference's acquisition grid dump (pcps_acquisition.cc:408-508): writes the
 * |R|^2 grid of PRN slot `prn_slot` for one host block into grid_host
 * (D rows of fft_size floats, Doppler-major).  Synchronous. */
int gsdr_acq_dump_grid(gsdr_acq* acq, const void* iq_host, uint32_t prn_slot, float* grid_host);
/* The narrow grid of make_two_steps for the same dump (d_narrow_grid,
 * pcps_acquisition.cc:743-746, written by dump_results :493-506): the |R|^2 grid of
 * PRN slot prn_slot over the num_doppler_bins_step2 rows centred on
 * doppler_center_hz (update_grid_doppler_wipeoffs_step2, :307-314) for one host
 * block, into grid_host (num_doppler_bins_step2 rows of fft_size floats).  Needs
 * gsdr_acq_set_step_two and num_doppler_bins_step2 <= the handle's Doppler bins.
 * Synchronous. */
int gsdr_acq_dump_grid_step_two(gsdr_acq* acq, const void* iq_host, uint32_t prn_slot, float doppler_center_hz,
    float* grid_host);

/* make_two_steps (pcps_acquisition.cc:298-314, :717-773, :781-800, :894-909;
 * Acq_Conf second_nbins / second_doppler_step / pfa_second_step, acq_conf.cc:63-76).
 * After a positive first step the reference searches the NEXT block on a narrow
 * grid of num_doppler_bins_step2 bins spaced doppler_step2 Hz around the coarse
 * Acq_doppler_hz (float arithmetic, no doppler_bias), with its own threshold
 * (pfa2 and the narrow bin count; pfa2 outside (0,1] means pfa as in Acq_Conf)
 * and, for CFAR, the first step's input power (d_input_power is not recomputed
 * in step two, :530-540).  set_step_two configures the narrow grid for the
 * handle; run_step_two runs it for nsel PRN slots of the current batch over one
 * attempt (max_dwells blocks) of host IQ, prn_slots[i] with centre
 * doppler_center_hz[i] (the coarse Acq_doppler_hz) and coarse_input_power[i]
 * (the coarse result's input_power; ignored by the peak-ratio statistic).
 * out[i]: the step-two Gnss_Synchro fields (doppler_hz from the narrow grid,
 * :539) and the decision against the step-two threshold.  Synchronous. */
int gsdr_acq_set_step_two(gsdr_acq* acq, uint32_t num_doppler_bins_step2, float doppler_step2, float pfa2);
int gsdr_acq_get_step_two_threshold(const gsdr_acq* acq, float* threshold);
int gsdr_acq_run_step_two(gsdr_acq* acq, const void* iq_host, uint32_t nsel, const uint32_t* prn_slots,
    const float* doppler_center_hz, const float* coarse_input_power, uint64_t stamp, gsdr_acq_result* out);

/* Stage profiling with HIP events recorded on the launch stream (observability,
 * the role of the reference's per-block timing prints).  When enabled, every
 * gsdr_acq_run / gsdr_acq_run_device call records device time per stage:
 * [0] forward FFT (x .* w_d), [1] fused correlate (code product + inverse FFT +
 * |.|^2 + row statistics), [2] grid reduction, [3] second-peak pass.
 * gsdr_acq_read_profile synchronises, returns the sums since the last read
 * (milliseconds) and the number of launches per stage, and resets them. */
int gsdr_acq_set_profiling(gsdr_acq* acq, int enable);
int gsdr_acq_read_profile(gsdr_acq* acq, double* stage_ms, uint32_t* launches);
/* The same, plus per stage the busy time: the union of its launches' [start, end)
 * intervals (stage_busy_ms may be NULL) -- the stage's wall time when launches of
 * the handle overlap (runs issued on several streams); stage_ms / launches then
 * over-counts it. */
int gsdr_acq_read_profile_ex(gsdr_acq* acq, double* stage_ms, uint32_t* launches, double* stage_busy_ms);
/* The recorded launches of one stage (0 forward, 1 correlate, 2 reduce/argmax,
 * 3 second peak) as [start, end) in ms against the caller's hipEvent_t ref_event
 * (recorded on the same device before them), so the busy time of one stage over
 * several handles -- chains on their own streams -- is the union of all their
 * intervals.  *n = the stage's launch count (entries beyond max_n not written).
 * Read before gsdr_acq_read_profile[_ex], which releases the records. */
int gsdr_acq_read_profile_intervals(gsdr_acq* acq, const void* ref_event, int stage, double* start_ms, double* end_ms,
    uint32_t max_n, uint32_t* n);

/* Debug/verification: device forward spectrum for one host block,
 * D rows x fft_size complex<float> (= FFT(x .* w_d)). */
int gsdr_acq_dump_spectra(gsdr_acq* acq, const void* iq_host, float* spectra_host);

/* ======================================================================== */
/* Tracking multicorrelator (Cpu_Multicorrelator_Real_Codes / Cpu_Multicorrelator) */
/* ======================================================================== */

typedef struct gsdr_corr gsdr_corr;

/* One correlation request: the 6 NCO parameters of
 * Carrier_wipeoff_multicorrelator_resampler (cpu_multicorrelator_real_codes.cc:103-126),
 * in the units dll_pll_veml_tracking passes them (do_correlation_step,
 * dll_pll_veml_tracking.cc:1064-1089): code terms already multiplied by samples/chip. */
typedef struct gsdr_corr_job
{
    int32_t channel;              /* correlator slot holding code + taps */
    int32_t n_samples;            /* signal_length_samples */
    int64_t sample_offset;        /* first input item of this job within the IQ buffer */
    float rem_carr_phase_rad;
    float carr_phase_step_rad;
    float carr_phase_rate_step_rad;
    float rem_code_phase_chips;
    float code_phase_step_chips;
    float code_phase_rate_step_chips;
} gsdr_corr_job;

/* init(max_signal_length_samples, n_correlators) for max_channels slots. */
int gsdr_corr_create(int device, int max_channels, int max_len, int max_taps, gsdr_corr** out);
void gsdr_corr_destroy(gsdr_corr* corr);

/* set_local_code_and_taps (cpu_multicorrelator_real_codes.cc:53-63); unlike the
 * reference (which keeps the caller's pointers) the code and shifts are copied
 * to the device, so the caller's arrays need not outlive the call. */
int gsdr_corr_set_local_code_and_taps(gsdr_corr* corr, int channel, int code_length_chips, const float* code,
    const float* shifts_chips, int n_taps);
/* Cpu_Multicorrelator::set_local_code_and_taps (complex replicas, cpu_multicorrelator.cc:54-62). */
int gsdr_corr_set_local_code_and_taps_complex(gsdr_corr* corr, int channel, int code_length_chips,
    const float* code_cf32, const float* shifts_chips, int n_taps);
/* set_high_dynamics_resampler (cpu_multicorrelator_real_codes.cc:161-165). */
int gsdr_corr_set_high_dynamics_resampler(gsdr_corr* corr, int channel, int enable);
/* Float association of the code-phase index (GSDR_ASSOC_*), default GSDR_ASSOC_AVX. */
int gsdr_corr_set_resampler_assoc(gsdr_corr* corr, int assoc);

/* Synchronous drop-in for one channel: Carrier_wipeoff_multicorrelator_resampler
 * (7-argument form) on host samples; writes n_taps complex<float> to corr_out_host.
 * item_type selects gr_complex or cshort input. */
int gsdr_corr_run(gsdr_corr* corr, int channel, const void* sig_in_host, int item_type, float rem_carr_phase_rad,
    float carr_phase_step_rad, float carr_phase_rate_step_rad, float rem_code_phase_chips,
    float code_phase_step_chips, float code_phase_rate_step_chips, int signal_length_samples, float* corr_out_host);

/* Batched form: njobs jobs over one device IQ buffer (iq_dev, iq_items items of
 * item_type).  Writes, for job j, n_taps(channel) complex<float> at
 * out_dev + 2*j*max_taps.  jobs_host is copied; asynchronous on stream. */
int gsdr_corr_run_batch(gsdr_corr* corr, const gsdr_corr_job* jobs_host, int njobs, const void* iq_dev,
    int item_type, int64_t iq_items, float* out_dev, void* stream);

/* Same, with the job table already in device memory (graph-capturable). */
int gsdr_corr_run_batch_device(gsdr_corr* corr, const gsdr_corr_job* jobs_dev, int njobs, const void* iq_dev,
    int item_type, int64_t iq_items, float* out_dev, void* stream);

/* Multi-epoch schedule: n_epochs consecutive batches of jobs_per_epoch jobs
 * (jobs_dev holds n_epochs*jobs_per_epoch jobs, epoch-major).  Epoch e is one
 * launch queued behind epoch e-1 on the stream — the launch order a tracking
 * loop imposes — issued from native code.  Output of job j of epoch e at
 * out_dev + 2*(e*jobs_per_epoch + j)*max_taps. */
int gsdr_corr_run_epochs(gsdr_corr* corr, const gsdr_corr_job* jobs_dev, int jobs_per_epoch, int n_epochs,
    const void* iq_dev, int item_type, int64_t iq_items, float* out_dev, void* stream);

/* Kernel-time profiling with HIP events (see gsdr_acq_set_profiling). */
int gsdr_corr_set_profiling(gsdr_corr* corr, int enable);
int gsdr_corr_read_profile(gsdr_corr* corr, double* kernel_ms, uint32_t* launches);

/* Debug/verification: the resampled code indices of one channel, as the
 * kernel computes them (n_taps rows x n samples int32, host). */
int gsdr_corr_dump_indices(gsdr_corr* corr, int channel, float rem_code_phase_chips, float code_phase_step_chips,
    int n, int32_t* idx_host);

/* ======================================================================== */
/* Tracking — device-resident DLL/PLL loop (dll_pll_veml_tracking)           */
/* ======================================================================== */
/*
 * Replaces the per-epoch work of dll_pll_veml_tracking::general_work
 * (src/algorithms/tracking/gnuradio_blocks/dll_pll_veml_tracking.cc:1784-2152):
 * do_correlation_step (:1064-1089), run_dll_pll (:1092-1179),
 * update_tracking_vars (:1216-1287), cn0_and_tracking_lock_status (:970-1056),
 * the bit-synchronisation preamble search (acquire_secondary, :923-967) and the
 * state machine (states 2 and 4).  One handle owns a pool of channels; a launch
 * advances every active channel by up to max_epochs general_work calls over a
 * device-resident IQ buffer without returning to the host (one workgroup per
 * channel loops over its epochs: the tracking loop is sequential in time per
 * channel, parallel across channels).
 */
typedef struct gsdr_trk gsdr_trk;

#define GSDR_SIGNAL_GPS_1C 0 /* GPS L1 C/A (dll_pll_veml_tracking.cc:170-191) */
#define GSDR_SIGNAL_GAL_1B 1 /* Galileo E1 OS, VEML 5 taps, pilot (E1C) or data (E1B) tracking (:258-290) */
#define GSDR_SIGNAL_BDS_B1 2 /* BeiDou B1I D1 (NH secondary code) / D2 GEO (preamble) (:391-411, :762-795) */

/* Mirrors Dll_Pll_Conf (src/algorithms/tracking/libs/dll_pll_conf.h:30-84);
 * gsdr_trk_conf_default() fills the reference defaults (incl. the gflags
 * defaults gnss_sdr_flags.cc:45-54 for cn0_samples, cn0_min, max_lock_fail,
 * max_carrier_lock_fail and carrier_lock_th). */
typedef struct gsdr_trk_conf
{
    double fs_in;
    double carrier_lock_th;
    uint32_t vector_length; /* correlation length; 0 -> round(fs_in / 1000) (gps_l1_ca_dll_pll_tracking.cc:42) */
    int32_t signal;         /* GSDR_SIGNAL_* */
    int32_t item_type;      /* GSDR_ITEM_* */
    uint32_t max_channels;
    float fll_bw_hz;
    float pll_bw_hz;
    float dll_bw_hz;
    float pll_bw_narrow_hz;
    float dll_bw_narrow_hz;
    float early_late_space_chips;
    float very_early_late_space_chips;
    float early_late_space_narrow_chips;
    float very_early_late_space_narrow_chips;
    float cn0_smoother_alpha;
    float carrier_lock_test_smoother_alpha;
    uint32_t pull_in_time_s;
    uint32_t bit_synchronization_time_limit_s;
    int32_t pll_filter_order;
    int32_t dll_filter_order;
    int32_t extend_correlation_symbols; /* coherent symbols per correlation after bit sync (state 3, :1989-2026) */
    int32_t cn0_samples;
    int32_t cn0_smoother_samples;
    int32_t carrier_lock_test_smoother_samples;
    int32_t cn0_min;
    int32_t max_code_lock_fail;
    int32_t max_carrier_lock_fail;
    int32_t enable_fll_pull_in;
    int32_t enable_fll_steady_state;
    int32_t carrier_aiding;
    int32_t high_dyn;    /* Dll_Pll_Conf::high_dyn: high-dynamics resampler/rotator + carrier/code rate
                            estimates from the step histories (dll_pll_veml_tracking.cc:1232-1284) */
    int32_t track_pilot; /* Dll_Pll_Conf::track_pilot (default 1); forced 0 for GPS L1 C/A and BeiDou B1I */
    uint32_t smoother_length; /* Dll_Pll_Conf::smoother_length (default 10, at most 32): histories of 2x that */
} gsdr_trk_conf;

/* One general_work call of one channel (written for every call that ran a
 * correlation or changed state).  Gnss_Synchro fields as general_work fills them
 * (:2000-2017, :2121-2127) plus the loop state after the call. */
typedef struct gsdr_trk_epoch
{
    uint64_t sample_counter;       /* nitems_read(0) at the start of the call */
    int32_t state;                 /* d_state at the start of the call */
    int32_t consumed;              /* consume_each() count */
    float taps[10];                /* correlator outputs of the call: E,P,L (3 taps) or VE,E,P,L,VL */
    float rem_carr_phase_rad;      /* after the call */
    int32_t flags;                 /* GSDR_TRK_F_* */
    double carrier_doppler_hz;     /* Carrier_Doppler_hz */
    double code_freq_chips;
    double rem_code_phase_samples; /* Code_phase_samples */
    double acc_carrier_phase_rad;  /* Carrier_phase_rads */
    double cn0_db_hz;              /* CN0_dB_hz */
    double carrier_lock_test;
    double prompt_i;               /* Prompt_I (valid output only) */
    double prompt_q;               /* Prompt_Q (valid output only) */
    double evm;                    /* EVM (fork indicator, :1027-1053) */
    float data_prompt[2];          /* pilot tracking: the data-component prompt of the call (d_Prompt_Data[0]) */
    float carrier_rate;            /* high_dyn: (float)d_carrier_phase_rate_step_rad after the call [rad/sample^2] */
    float code_rate;               /* high_dyn: (float)d_code_phase_rate_step_chips after the call [chips/sample^2] */
    /* log_data (dll_pll_veml_tracking.cc:1403-1500), valid when flags has GSDR_TRK_F_LOGGED: the
     * accumulator magnitudes |VE|, |E|, |P|, |L|, |VL| (VE/VL 0 without VEML) and the loop
     * errors as the dump writes them (static_cast<float> of the double members) */
    float log_accu[5];
    float carr_phase_error_hz, carr_error_filt_hz, code_error_chips, code_error_filt_chips;
    int32_t reserved;              /* 0 (keeps the record free of padding bytes) */
} gsdr_trk_epoch;

#define GSDR_TRK_F_VALID_OUTPUT 1 /* Flag_valid_symbol_output: a Gnss_Synchro was emitted */
#define GSDR_TRK_F_LOSS_OF_LOCK 2 /* event 3 (loss of lock), channel back to state 0 */
#define GSDR_TRK_F_PLL_180 4      /* Flag_PLL_180_deg_phase_locked */
#define GSDR_TRK_F_BIT_SYNC 8     /* preamble / bit synchronisation locked in this call (2 -> 4) */
#define GSDR_TRK_F_OVERRUN 16     /* with LOSS_OF_LOCK: the channel's next call starts before the oldest
                                     input item given (the ring moved past a stalled channel); the
                                     record carries the channel's position, the channel is in state 0 */
#define GSDR_TRK_F_LOGGED 32      /* the reference calls log_data() for this call (state 2 locked; states
                                     3/4 with a completed data symbol): the record's log_* fields are set */

void gsdr_trk_conf_default(gsdr_trk_conf* conf);
int gsdr_trk_create(int device, const gsdr_trk_conf* conf, gsdr_trk** out);
void gsdr_trk_destroy(gsdr_trk* trk);

/* start_tracking (:640-882) for channel ch with the acquisition results of
 * Gnss_Synchro (Acq_delay_samples, Acq_doppler_hz, Acq_samplestamp_samples) and
 * the PRN's tracking code replica (code_samples = samples_per_chip * code length
 * floats, e.g. gps_l1_ca_code_gen_float), followed by the state-1 pull-in call
 * (:1813-1844) executed at input position nitems_read.  *first_sample receives
 * the absolute input index of the first correlation (nitems_read + offset). */
int gsdr_trk_start(gsdr_trk* trk, int ch, uint32_t prn, const float* code, int code_samples,
    double acq_delay_samples, double acq_doppler_hz, uint64_t acq_samplestamp, uint64_t nitems_read,
    uint64_t* first_sample);
/* Pilot tracking (track_pilot, Galileo E1): the data component's replica for the
 * extra prompt correlator (d_correlator_data_cpu.set_local_code_and_taps,
 * dll_pll_veml_tracking.cc:681-689, e.g. galileo_e1_code_gen_sinboc11_float of
 * E1B), code_samples floats.  Call before gsdr_trk_start for that channel. */
int gsdr_trk_set_data_code(gsdr_trk* trk, int ch, const float* data_code, int code_samples);
/* stop_tracking: channel to state 0 (standby). */
int gsdr_trk_stop(gsdr_trk* trk, int ch);
/* msg_handler_telemetry_to_trk with tlm_event 1 (dll_pll_veml_tracking.cc:614-637,
 * port registered :142-147): a telemetry fault forces d_carrier_lock_fail_counter to
 * 200000, so the channel's next lock check past the CN0 fill (states 2 / 4) reports
 * the loss of lock (GSDR_TRK_F_LOSS_OF_LOCK).  Takes effect at the channel's next
 * call on the device (synchronous; ordered after the handle's last launch). */
int gsdr_trk_force_loss_of_lock(gsdr_trk* trk, int ch);

/* Advance every channel in states 2..4 by up to max_epochs general_work calls
 * over iq_dev, which holds iq_items items whose first item is absolute input
 * sample iq_first_sample.  A channel stops early when its next call would read
 * past the buffer.  out_dev: max_channels * max_epochs records, channel-major
 * (record e of channel c at c*max_epochs + e); n_out_dev: per-channel record
 * count (device).  Asynchronous on stream (NULL = the handle's own stream). */
int gsdr_trk_run_device(gsdr_trk* trk, const void* iq_dev, uint64_t iq_first_sample, uint64_t iq_items,
    uint32_t max_epochs, gsdr_trk_epoch* out_dev, uint32_t* n_out_dev, void* stream);

/* Ring form: every active channel advances by up to max_epochs calls over the
 * ring's newest contiguous window (gsdr_stream_span); a channel whose next call
 * needs items not pushed yet stops and continues on a later call, so pushing the
 * stream in any chunking gives the records of one contiguous run.  Asynchronous on
 * stream (NULL = the handle's own), ordered after the ring's pushes and before the
 * pushes that would overwrite the window. */
int gsdr_trk_run_stream(gsdr_trk* trk, gsdr_stream* ring, uint32_t max_epochs, gsdr_trk_epoch* out_dev,
    uint32_t* n_out_dev, void* stream);

/* Ring form with the records copied back to the host (synchronous; the
 * handle's own stream and record buffers): the tracking pool service's call. */
int gsdr_trk_run_stream_host(gsdr_trk* trk, gsdr_stream* ring, uint32_t max_epochs, gsdr_trk_epoch* out_host,
    uint32_t* n_out_host);

/* Asynchronous ring form for a host consumer (the pooled tracking blocks of
 * dll_pll_veml_tracking_pool_mi355x, which replace the per-channel general_work
 * round trips of dll_pll_veml_tracking.cc:1784-2152): gsdr_trk_run_stream on the
 * handle's stream into the handle's own submission buffers, the records and counts
 * copied into pinned host memory behind it; returns without waiting.  Up to two
 * submissions in flight (the second runs behind the first on the handle's stream, so
 * the GPU does not idle while the host collects); gsdr_trk_collect copies out the
 * oldest: out_host holds max_channels *
 * max_epochs records (channel-major; only the first n_out_host[c] of channel c are
 * written), n_out_host max_channels counts, *max_epochs
 * (may be NULL) the submission's max_epochs; wait != 0 waits for the copy, wait == 0
 * returns 1 without copying while it is in flight.  Submits on one handle are
 * serialised (each keeps its slot while it launches); a collect may run beside a
 * submit and sees only submissions that returned GSDR_OK. */
int gsdr_trk_submit_stream(gsdr_trk* trk, gsdr_stream* ring, uint32_t max_epochs);
int gsdr_trk_collect(gsdr_trk* trk, int wait, gsdr_trk_epoch* out_host, uint32_t* n_out_host, uint32_t* max_epochs);

/* Host form of the same call (synchronous): copies the records back. */
int gsdr_trk_run(gsdr_trk* trk, const void* iq_host, uint64_t iq_first_sample, uint64_t iq_items,
    uint32_t max_epochs, gsdr_trk_epoch* out_host, uint32_t* n_out_host);

/* Channel snapshot: current state, next input index, Doppler and CN0. */
int gsdr_trk_get_channel(gsdr_trk* trk, int ch, int32_t* state, uint64_t* next_sample, double* carrier_doppler_hz,
    double* cn0_db_hz);

/* Device-side copy of every channel's loop state into / out of snapshot slot
 * `slot` (0 or 1); asynchronous on stream.  Lets a caller replay the same input
 * span from the same loop state (benchmarks, what-if re-tracking). */
int gsdr_trk_save_state(gsdr_trk* trk, int slot, void* stream);
int gsdr_trk_restore_state(gsdr_trk* trk, int slot, void* stream);

/* Kernel-time profiling with HIP events (see gsdr_acq_set_profiling). */
int gsdr_trk_set_profiling(gsdr_trk* trk, int enable);

/* Compute-unit partitioning (MI355X: 256 CUs in 8 XCDs).  Recreates the handle's
 * own stream (the one used when a call passes stream = NULL) restricted to the CUs
 * whose bits are set in mask[0..n_words) -- bit i selects CU i/8 of XCD i%8
 * (hipExtStreamCreateWithCUMask numbering).  A latency-bound tracking pool can so
 * own a few CUs while the throughput-bound acquisition grid fills the rest.
 * n_words = 0 restores an unrestricted stream. */
int gsdr_acq_set_cu_mask(gsdr_acq* acq, const uint32_t* mask, int n_words);
int gsdr_trk_set_cu_mask(gsdr_trk* trk, const uint32_t* mask, int n_words);
int gsdr_trk_read_profile(gsdr_trk* trk, double* kernel_ms, uint32_t* launches);

#ifdef __cplusplus
}
#endif

#endif /* GSDR_H */
