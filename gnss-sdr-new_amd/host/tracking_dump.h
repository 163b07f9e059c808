// The tracking block's binary dump (dll_pll_veml_tracking.cc:565-597 file naming,
// :1733-1760 per-channel file, :1403-1500 log_data record) written on the host from
// the engine's gsdr_trk_epoch records: the engine flags the calls at which the
// reference calls log_data() (GSDR_TRK_F_LOGGED) and carries the accumulator
// magnitudes and loop errors of that point, so the file holds the same 108-byte
// records in the same order.  save_matfile (:1511-1729, run by the destructor when
// dump_mat, :884-906) converts the channel's .dat into <stem><channel>.mat with the
// reference's 25 variable names, classes and 1 x epochs dimensions, as a Level-5
// MAT-file (Mat5Writer; the reference's matio writes MAT 7.3, which needs HDF5).
#ifndef GSDR_HOST_TRACKING_DUMP_H
#define GSDR_HOST_TRACKING_DUMP_H

#include <cstdint>
#include <fstream>
#include <string>

#include "gsdr.h"

class TrackingDump
{
public:
    static constexpr size_t kRecordBytes = 108;

    // constructor part (:565-597): path and stem of dump_filename, the stem's
    // extension removed, "trk_channel_" for an empty stem; the directory is
    // created.  Returns false (dump off) when it cannot be created.
    bool configure(const std::string& dump_filename);
    // set_channel (:1733-1760): open <stem><channel>.dat if not open yet
    bool open(uint32_t channel);
    // start_tracking's acquisition values written into every record (:1496-1499)
    void set_acquisition(uint32_t prn, double acq_code_phase_samples, double acq_carrier_doppler_hz);
    // d_acq_code_phase_samples after the pull-in (:1817-1828) for signal GSDR_SIGNAL_*
    static double pull_in_code_phase(int32_t signal, double fs_in, uint64_t nitems_read, uint64_t acq_sample_stamp,
        double acq_delay_samples);
    // one record if the call logged (GSDR_TRK_F_LOGGED); veml: taps are VE,E,P,L,VL
    void write(const gsdr_trk_epoch& r, double fs_in, bool veml, bool track_pilot);
    // the record bytes alone (no file): out must hold kRecordBytes
    static void encode(const gsdr_trk_epoch& r, double fs_in, bool veml, bool track_pilot, uint32_t prn,
        double acq_code_phase_samples, double acq_carrier_doppler_hz, char* out);
    // close the .dat and convert <stem><channel>.dat of the last set_channel into
    // <stem><channel>.mat (save_matfile); false when the .dat cannot be read
    bool save_matfile();
    bool is_open() const { return file_.is_open(); }
    const std::string& stem() const { return stem_; }
    const std::string& path() const { return path_; }

private:
    std::string stem_;
    std::string path_;
    std::ofstream file_;
    uint32_t channel_{0};  // d_channel: save_matfile reads the file of the last set_channel
    uint32_t prn_{0};
    double acq_code_phase_{0.0};
    double acq_doppler_{0.0};
};

#endif
