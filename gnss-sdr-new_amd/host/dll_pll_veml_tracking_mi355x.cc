#include "dll_pll_veml_tracking_mi355x.h"

#include <algorithm>
#include <iostream>
#include <stdexcept>
#include <string>

#include "gnss_replicas.h"

dll_pll_veml_tracking_mi355x::dll_pll_veml_tracking_mi355x(const Dll_Pll_Conf& conf, int32_t signal, int device)
    : d_conf(conf), d_signal(signal), d_device(device)
{
    const gsdr_trk_conf c = d_conf.to_engine(signal, 1);
    if (gsdr_trk_create(device, &c, &d_engine) != GSDR_OK)
        throw std::runtime_error(std::string("dll_pll_veml_tracking_mi355x: ") + gsdr_last_error());
    d_vector_length = d_conf.vector_length;
    if (d_conf.dump) d_dump.configure(d_conf.dump_filename);
    d_item_bytes = c.item_type == GSDR_ITEM_CSHORT ? 4 : (c.item_type == GSDR_ITEM_IBYTE ? 2 : 8);
    d_output = TrackingOutput(d_conf.fs_in, signal);
}

dll_pll_veml_tracking_mi355x::~dll_pll_veml_tracking_mi355x()
{
    // the destructor's .dat close and save_matfile (:884-906)
    if (d_conf.dump && d_conf.dump_mat) d_dump.save_matfile();
    gsdr_trk_destroy(d_engine);
}

void dll_pll_veml_tracking_mi355x::set_gnss_synchro(Gnss_Synchro* p_gnss_synchro)
{
    std::lock_guard<std::mutex> l(d_setlock);
    d_acquisition_gnss_synchro = p_gnss_synchro;
}

void dll_pll_veml_tracking_mi355x::set_channel(uint32_t channel)
{
    std::lock_guard<std::mutex> l(d_setlock);
    d_channel = channel;
    if (d_conf.dump) d_dump.open(channel);
}

void dll_pll_veml_tracking_mi355x::start_tracking()
{
    std::lock_guard<std::mutex> l(d_setlock);
    if (!d_acquisition_gnss_synchro) throw std::logic_error("dll_pll_veml_tracking_mi355x: set_gnss_synchro first");
    d_state = 1;
}

void dll_pll_veml_tracking_mi355x::stop_tracking()
{
    std::lock_guard<std::mutex> l(d_setlock);
    d_state = 0;
    d_fault_pending = false;
    gsdr_trk_stop(d_engine, 0);
}

void dll_pll_veml_tracking_mi355x::msg_handler_telemetry_to_trk(int tlm_event)
{
    if (tlm_event != 1) return;
    std::lock_guard<std::mutex> l(d_setlock);
    // d_carrier_lock_fail_counter = 200000 (:625): on the engine's channel while it
    // tracks; between start_tracking and the pull-in the engine's start (which
    // resets the counters, as start_tracking does at :836) comes first, so the
    // fault is applied right after it; in standby the next start_tracking resets it
    if (d_state == 2)
        {
            if (gsdr_trk_force_loss_of_lock(d_engine, 0) != GSDR_OK)
                std::cerr << "dll_pll_veml_tracking_mi355x: " << gsdr_last_error() << '\n';
        }
    else if (d_state == 1)
        d_fault_pending = true;
}

// The tracking replica of start_tracking (:661-700): GPS gps_l1_ca_code_gen_float,
// Galileo E1 galileo_e1_code_gen_sinboc11_float of E1-C when tracking the pilot
// (E1-B as the data-component replica) or of the channel's signal, BeiDou
// beidou_b1i_code_gen_float.
void dll_pll_veml_tracking_mi355x::load_codes(uint32_t prn, std::vector<float>& code)
{
    if (d_signal == GSDR_SIGNAL_GAL_1B)
        {
            const char sig[3] = {d_acquisition_gnss_synchro->Signal[0], d_acquisition_gnss_synchro->Signal[1], '\0'};
            if (d_conf.track_pilot)
                {
                    code = galileo_e1_code_gen_sinboc11_float("1C", prn);
                    const auto data = galileo_e1_code_gen_sinboc11_float(sig, prn);
                    if (gsdr_trk_set_data_code(d_engine, 0, data.data(), static_cast<int>(data.size())) != GSDR_OK)
                        throw std::runtime_error(std::string("dll_pll_veml_tracking_mi355x: ") + gsdr_last_error());
                }
            else
                code = galileo_e1_code_gen_sinboc11_float(sig, prn);
        }
    else if (d_signal == GSDR_SIGNAL_BDS_B1)
        code = beidou_b1i_code_gen_float(static_cast<int32_t>(prn), 0);
    else
        code = gps_l1_ca_code_gen_float(static_cast<int32_t>(prn), 0);
}

int dll_pll_veml_tracking_mi355x::work(const void* in, int ninput_items, uint64_t nitems_read, Gnss_Synchro* out,
    int* noutput, TrackingTags* tags)
{
    std::lock_guard<std::mutex> l(d_setlock);
    *noutput = 0;
    if (tags) tags->has_out = false;
    switch (d_state)
        {
        case 0:  // standby: consume at full throttle (:1806-1811)
            return ninput_items;
        case 1:
            {
                // pull-in (:1813-1844): align to the next code start after nitems_read
                std::vector<float> code;
                load_codes(d_acquisition_gnss_synchro->PRN, code);
                uint64_t first = 0;
                if (gsdr_trk_start(d_engine, 0, d_acquisition_gnss_synchro->PRN, code.data(), static_cast<int>(code.size()),
                        d_acquisition_gnss_synchro->Acq_delay_samples, d_acquisition_gnss_synchro->Acq_doppler_hz,
                        d_acquisition_gnss_synchro->Acq_samplestamp_samples, nitems_read, &first) != GSDR_OK)
                    {
                        std::cerr << "dll_pll_veml_tracking_mi355x: " << gsdr_last_error() << '\n';
                        d_state = 0;
                        if (d_events) d_events(3);
                        return 0;
                    }
                if (d_conf.dump)
                    d_dump.set_acquisition(d_acquisition_gnss_synchro->PRN,
                        TrackingDump::pull_in_code_phase(d_signal, d_conf.fs_in, nitems_read,
                            d_acquisition_gnss_synchro->Acq_samplestamp_samples,
                            d_acquisition_gnss_synchro->Acq_delay_samples),
                        d_acquisition_gnss_synchro->Acq_doppler_hz);
                d_state = 2;
                if (d_fault_pending)
                    {
                        d_fault_pending = false;
                        gsdr_trk_force_loss_of_lock(d_engine, 0);
                    }
                return static_cast<int>(first - nitems_read);
            }
        default:
            break;
        }
    // states 2..4: one general_work call of the engine over the forecast window
    if (ninput_items <= 0 || !in) return 0;
    const int n = std::min(ninput_items, forecast());
    uint32_t nrec = 0;
    if (gsdr_trk_run(d_engine, in, nitems_read, static_cast<uint64_t>(n), 1, &d_last, &nrec) != GSDR_OK)
        {
            // device error -> loss of lock, the reference's failure convention
            std::cerr << "dll_pll_veml_tracking_mi355x: " << gsdr_last_error() << '\n';
            d_state = 0;
            if (d_events) d_events(3);
            return 0;
        }
    if (nrec == 0) return 0;  // not enough input for the call: wait for more items
    if (d_record_sink) d_record_sink(d_last);
    if (d_conf.dump) d_dump.write(d_last, d_conf.fs_in, d_signal == GSDR_SIGNAL_GAL_1B, d_conf.track_pilot);
    const bool loss_of_lock = (d_last.flags & GSDR_TRK_F_LOSS_OF_LOCK) != 0;
    if (d_output.emit(d_last, *d_acquisition_gnss_synchro, nitems_read, out)) *noutput = 1;
    d_output.call_tags(tags, nitems_read, d_last.consumed, *noutput ? out : nullptr, d_nitems_written);
    d_nitems_written += static_cast<uint64_t>(*noutput);
    if (loss_of_lock)
        {
            d_state = 0;
            if (d_events) d_events(3);
        }
    return d_last.consumed;
}
