#include "dll_pll_conf.h"

#include <iostream>

#include "gnss_sdr_flags.h"

// dll_pll_conf.cc:24-28: the lock-detector defaults come from the gflags
Dll_Pll_Conf::Dll_Pll_Conf()
    : carrier_lock_th(FLAGS_carrier_lock_th),
      cn0_samples(FLAGS_cn0_samples),
      cn0_min(FLAGS_cn0_min),
      max_code_lock_fail(FLAGS_max_lock_fail),
      max_carrier_lock_fail(FLAGS_max_carrier_lock_fail)
{
    signal[0] = '1';
    signal[1] = 'C';
    signal[2] = '\0';
}

void Dll_Pll_Conf::SetFromConfiguration(const ConfigurationInterface* configuration, const std::string& role)
{
    item_type = configuration->property(role + ".item_type", item_type);
    if (item_type != "gr_complex" && item_type != "cshort" && item_type != "cbyte")
        {
            std::cerr << "Unknown item type: " << item_type << ". Set to gr_complex\n";
            item_type = "gr_complex";
        }
    const double fs_in_deprecated = configuration->property("GNSS-SDR.internal_fs_hz", fs_in);
    fs_in = configuration->property("GNSS-SDR.internal_fs_sps", fs_in_deprecated);
    high_dyn = configuration->property(role + ".high_dyn", high_dyn);
    dump = configuration->property(role + ".dump", dump);
    dump_filename = configuration->property(role + ".dump_filename", dump_filename);
    dump_mat = configuration->property(role + ".dump_mat", dump_mat);
    pll_bw_hz = configuration->property(role + ".pll_bw_hz", pll_bw_hz);
    if (FLAGS_pll_bw_hz != 0.0) pll_bw_hz = static_cast<float>(FLAGS_pll_bw_hz);  // :53-56
    pll_bw_narrow_hz = configuration->property(role + ".pll_bw_narrow_hz", pll_bw_narrow_hz);
    dll_bw_narrow_hz = configuration->property(role + ".dll_bw_narrow_hz", dll_bw_narrow_hz);
    dll_bw_hz = configuration->property(role + ".dll_bw_hz", dll_bw_hz);
    if (FLAGS_dll_bw_hz != 0.0) dll_bw_hz = static_cast<float>(FLAGS_dll_bw_hz);  // :60-63
    dll_filter_order = configuration->property(role + ".dll_filter_order", dll_filter_order);
    pll_filter_order = configuration->property(role + ".pll_filter_order", pll_filter_order);
    if (dll_filter_order < 1) dll_filter_order = 1;
    if (dll_filter_order > 3) dll_filter_order = 3;
    if (pll_filter_order < 2) pll_filter_order = 2;
    if (pll_filter_order > 3) pll_filter_order = 3;
    fll_filter_order = pll_filter_order == 2 ? 1 : 2;
    enable_fll_pull_in = configuration->property(role + ".enable_fll_pull_in", enable_fll_pull_in);
    enable_fll_steady_state = configuration->property(role + ".enable_fll_steady_state", enable_fll_steady_state);
    fll_bw_hz = configuration->property(role + ".fll_bw_hz", fll_bw_hz);
    pull_in_time_s = configuration->property(role + ".pull_in_time_s", pull_in_time_s);
    bit_synchronization_time_limit_s =
        configuration->property(role + ".bit_synchronization_time_limit_s", bit_synchronization_time_limit_s);
    early_late_space_chips = configuration->property(role + ".early_late_space_chips", early_late_space_chips);
    early_late_space_narrow_chips =
        configuration->property(role + ".early_late_space_narrow_chips", early_late_space_narrow_chips);
    very_early_late_space_chips = configuration->property(role + ".very_early_late_space_chips", very_early_late_space_chips);
    very_early_late_space_narrow_chips =
        configuration->property(role + ".very_early_late_space_narrow_chips", very_early_late_space_narrow_chips);
    extend_correlation_symbols = configuration->property(role + ".extend_correlation_symbols", extend_correlation_symbols);
    track_pilot = configuration->property(role + ".track_pilot", track_pilot);
    cn0_samples = configuration->property(role + ".cn0_samples", cn0_samples);
    cn0_min = configuration->property(role + ".cn0_min", cn0_min);
    max_code_lock_fail = configuration->property(role + ".max_lock_fail", max_code_lock_fail);
    max_carrier_lock_fail = configuration->property(role + ".max_carrier_lock_fail", max_carrier_lock_fail);
    carrier_lock_th = configuration->property(role + ".carrier_lock_th", carrier_lock_th);
    carrier_aiding = configuration->property(role + ".carrier_aiding", carrier_aiding);
    cn0_smoother_samples = configuration->property(role + ".cn0_smoother_samples", cn0_smoother_samples);
    cn0_smoother_alpha = configuration->property(role + ".cn0_smoother_alpha", cn0_smoother_alpha);
    smoother_length = configuration->property(role + ".smoother_length", smoother_length);
    if (smoother_length < 1) smoother_length = 1;
    carrier_lock_test_smoother_samples =
        configuration->property(role + ".carrier_lock_test_smoother_samples", carrier_lock_test_smoother_samples);
    carrier_lock_test_smoother_alpha =
        configuration->property(role + ".carrier_lock_test_smoother_alpha", carrier_lock_test_smoother_alpha);
}

gsdr_trk_conf Dll_Pll_Conf::to_engine(int32_t sig, uint32_t max_channels) const
{
    gsdr_trk_conf c;
    gsdr_trk_conf_default(&c);
    c.fs_in = fs_in;
    c.carrier_lock_th = carrier_lock_th;
    c.vector_length = vector_length;
    c.signal = sig;
    c.item_type = item_type == "cshort" ? GSDR_ITEM_CSHORT : (item_type == "cbyte" ? GSDR_ITEM_IBYTE : GSDR_ITEM_GR_COMPLEX);
    c.max_channels = max_channels;
    c.fll_bw_hz = fll_bw_hz;
    c.pll_bw_hz = pll_bw_hz;
    c.dll_bw_hz = dll_bw_hz;
    c.pll_bw_narrow_hz = pll_bw_narrow_hz;
    c.dll_bw_narrow_hz = dll_bw_narrow_hz;
    c.early_late_space_chips = early_late_space_chips;
    c.very_early_late_space_chips = very_early_late_space_chips;
    c.early_late_space_narrow_chips = early_late_space_narrow_chips;
    c.very_early_late_space_narrow_chips = very_early_late_space_narrow_chips;
    c.cn0_smoother_alpha = cn0_smoother_alpha;
    c.carrier_lock_test_smoother_alpha = carrier_lock_test_smoother_alpha;
    c.pull_in_time_s = pull_in_time_s;
    c.bit_synchronization_time_limit_s = bit_synchronization_time_limit_s;
    c.pll_filter_order = pll_filter_order;
    c.dll_filter_order = dll_filter_order;
    c.extend_correlation_symbols = extend_correlation_symbols;
    c.cn0_samples = cn0_samples;
    c.cn0_smoother_samples = cn0_smoother_samples;
    c.carrier_lock_test_smoother_samples = carrier_lock_test_smoother_samples;
    c.cn0_min = cn0_min;
    c.max_code_lock_fail = max_code_lock_fail;
    c.max_carrier_lock_fail = max_carrier_lock_fail;
    c.enable_fll_pull_in = enable_fll_pull_in ? 1 : 0;
    c.enable_fll_steady_state = enable_fll_steady_state ? 1 : 0;
    c.carrier_aiding = carrier_aiding ? 1 : 0;
    c.high_dyn = high_dyn ? 1 : 0;
    c.track_pilot = track_pilot ? 1 : 0;
    c.smoother_length = smoother_length;
    return c;
}
