#include "tracking_output.h"

#include <cmath>

int32_t tracking_correlation_length_ms(int32_t signal)
{
    return signal == GSDR_SIGNAL_GAL_1B ? 4 : 1;
}

bool TrackingOutput::emit(const gsdr_trk_epoch& r, const Gnss_Synchro& acq, uint64_t nitems_read,
    Gnss_Synchro* out) const
{
    const bool loss_of_lock = (r.flags & GSDR_TRK_F_LOSS_OF_LOCK) != 0;
    if (!(r.flags & GSDR_TRK_F_VALID_OUTPUT) && !loss_of_lock) return false;
    // current_synchro_data = *d_acquisition_gnss_synchro (:1878, :2040, :2003, :2056)
    Gnss_Synchro s = acq;
    if (!loss_of_lock)
        {
            // :2004-2017 / :2057-2070 (Prompt from d_P_data_accu, as the engine reports it)
            s.Prompt_I = r.prompt_i;
            s.Prompt_Q = r.prompt_q;
            s.Code_phase_samples = r.rem_code_phase_samples;
            s.Carrier_phase_rads = r.acc_carrier_phase_rad;
            s.Carrier_Doppler_hz = r.carrier_doppler_hz;
            s.CN0_dB_hz = r.cn0_db_hz;
            s.correlation_length_ms = corr_ms_;
            s.EVM = r.evm;
        }
    // :2121-2127
    s.fs = static_cast<int64_t>(fs_);
    s.Tracking_sample_counter = nitems_read;
    s.Flag_valid_symbol_output = !loss_of_lock;
    s.Flag_PLL_180_deg_phase_locked = (r.flags & GSDR_TRK_F_PLL_180) != 0;
    *out = s;
    return true;
}

void TrackingOutput::call_tags(TrackingTags* tags, uint64_t nitems_read, int32_t consumed, const Gnss_Synchro* out,
    uint64_t nitems_written)
{
    if (tags)
        {
            tags->has_out = false;
            // get_tags_in_range(0, nitems_read, nitems_read + d_current_prn_length_samples)
            // (:2088-2116): d_current_prn_length_samples is the call's consume_each count
            const uint64_t end = nitems_read + static_cast<uint64_t>(consumed > 0 ? consumed : 0);
            for (int i = 0; i < tags->n_in; ++i)
                {
                    const GnssTimeTag& t = tags->in[i];
                    if (t.offset < nitems_read || t.offset >= end) continue;
                    last_ = t.time;
                    last_offset_ = t.offset;
                    waiting_ = true;
                }
        }
    if (!out || !waiting_) return;
    // :2131-2146: the kept tag advanced by the (signed) sample distance to the output
    const uint64_t a = out->Tracking_sample_counter, b = last_offset_;
    const int64_t diff = a > b ? static_cast<int64_t>(a - b) : -static_cast<int64_t>(b - a);
    double intpart;
    last_.tow_ms_fraction = last_.tow_ms_fraction + std::modf(1000.0 * static_cast<double>(diff) / fs_, &intpart);
    if (tags)
        {
            tags->has_out = true;
            tags->out.offset = nitems_written + 1;
            tags->out.time.week = last_.week;
            tags->out.time.tow_ms = last_.tow_ms + static_cast<int>(intpart);
            tags->out.time.tow_ms_fraction = last_.tow_ms_fraction;
            tags->out.time.rx_time = static_cast<double>(out->Tracking_sample_counter) / fs_;
        }
    waiting_ = false;
}
