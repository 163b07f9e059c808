// TrackingInterface mirror (src/core/interfaces/tracking_interface.h:47-54) on the
// flowgraph-free GNSSBlockInterface subset (gnss_block_interface.h:68-102), as
// acquisition_interface.h does for AcquisitionInterface.
#ifndef GSDR_HOST_TRACKING_INTERFACE_H
#define GSDR_HOST_TRACKING_INTERFACE_H

#include <cstddef>
#include <string>

#include "gnss_synchro.h"

class TrackingInterface
{
public:
    virtual ~TrackingInterface() = default;
    // GNSSBlockInterface, flowgraph-free subset
    virtual std::string role() = 0;
    virtual std::string implementation() = 0;
    virtual size_t item_size() = 0;

    virtual void start_tracking() = 0;
    virtual void stop_tracking() = 0;
    virtual void set_gnss_synchro(Gnss_Synchro* gnss_synchro) = 0;
    virtual void set_channel(unsigned int channel) = 0;
};

#endif
