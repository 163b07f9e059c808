// Registration of the MI355X blocks: the GetAcqBlock / GetTrkBlock string
// switches of GNSSBlockFactory (src/core/receiver/gnss_block_factory.cc:1335-1519,
// :1522-1682) for the implementation names this engine provides, and the
// deterministic channel -> GPU map that replaces the CUDA path's per-instance
// rand() % num_devices (src/algorithms/tracking/libs/cuda_multicorrelator.cu:135-155).
//
// A maintainer adds the `if (implementation == "..._MI355X")` branches to the
// reference factory; here the same switch is a free function so
// the adapters can be built from a .conf without GNU Radio.
#ifndef GSDR_HOST_GNSS_BLOCK_FACTORY_MI355X_H
#define GSDR_HOST_GNSS_BLOCK_FACTORY_MI355X_H

#include <memory>
#include <string>

#include "acquisition_interface.h"
#include "configuration.h"
#include "tracking_interface.h"

namespace gsdr_factory
{
// GPU of channel `channel`: `<role>.device` when the configuration sets it, else
// channel % G with G = GNSS-SDR.mi355x_devices (default: every visible device).
// Channels are independent, so this static map is the whole
// multi-GPU scheme: no collective, each GPU ingests the stream for its channels.
int device_for_channel(const ConfigurationInterface* configuration, const std::string& role, int channel);

// nullptr when the implementation name is not an MI355X block (the reference
// factory then falls through to its own switch).
std::unique_ptr<AcquisitionInterface> GetAcqBlock(const ConfigurationInterface* configuration, const std::string& role,
    unsigned int in_streams, unsigned int out_streams, int channel = 0);
std::unique_ptr<TrackingInterface> GetTrkBlock(const ConfigurationInterface* configuration, const std::string& role,
    unsigned int in_streams, unsigned int out_streams, int channel = 0);
}  // namespace gsdr_factory

#endif
