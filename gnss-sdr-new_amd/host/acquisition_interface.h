// AcquisitionInterface mirror (src/core/interfaces/acquisition_interface.h:50-70)
// without the GNU Radio parts of GNSSBlockInterface (connect/get_left_block),
// which need a flowgraph this engine does not rebuild.
#ifndef GSDR_HOST_ACQUISITION_INTERFACE_H
#define GSDR_HOST_ACQUISITION_INTERFACE_H

#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

#include "gnss_synchro.h"

class ChannelFsm;

class AcquisitionInterface
{
public:
    virtual ~AcquisitionInterface() = default;
    // GNSSBlockInterface (gnss_block_interface.h:68-102), flowgraph-free subset
    virtual std::string role() = 0;
    virtual std::string implementation() = 0;
    virtual size_t item_size() = 0;

    virtual void set_gnss_synchro(Gnss_Synchro* gnss_synchro) = 0;
    virtual void set_channel(unsigned int channel_id) = 0;
    virtual void set_channel_fsm(std::weak_ptr<ChannelFsm> channel_fsm) = 0;
    virtual void set_threshold(float threshold) = 0;
    virtual void set_doppler_max(unsigned int doppler_max) = 0;
    virtual void set_doppler_step(unsigned int doppler_step) = 0;
    virtual void set_doppler_center(int doppler_center __attribute__((unused))) {}
    virtual void init() = 0;
    virtual void set_local_code() = 0;
    virtual void set_state(int state) = 0;
    virtual signed int mag() = 0;
    virtual void reset() = 0;
    virtual void stop_acquisition() = 0;
    virtual void set_resampler_latency(uint32_t latency_samples) = 0;
};

#endif
