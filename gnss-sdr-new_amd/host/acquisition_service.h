// One GPU acquisition grid serving every channel's acquisition requests
// (SURVEY.md §8f rank 2).
//
// In the reference every channel owns a pcps_acquisition block that searches one
// PRN per call over the shared sample stream (GNSSFlowgraph::connect wires the
// same signal-conditioner output to all acquisition blocks,
// src/core/receiver/gnss_flowgraph.cc:1796-1901; the channel FSM arms one
// acquisition per channel, src/algorithms/channel/libs/channel_fsm.cc:80-135).
// Here the channels post requests (PRN + replica + decision callback) to one
// service; each time a block of consumed_samples items is complete the service
// runs ONE batched acquisition_core over all pending PRNs (gsdr_acq_run with
// P = number of requests) and answers each request with its Gnss_Synchro
// acquisition fields and the positive/negative event of
// pcps_acquisition::acquisition_core (:781-829, single dwell).
#ifndef GSDR_HOST_ACQUISITION_SERVICE_H
#define GSDR_HOST_ACQUISITION_SERVICE_H

#include <complex>
#include <cstdint>
#include <functional>
#include <mutex>
#include <vector>

#include "acq_conf.h"
#include "gsdr.h"

class AcquisitionService
{
public:
    // result: the engine's record for this request; positive: statistic > threshold
    using Callback = std::function<void(uint32_t channel, const gsdr_acq_result& result, bool positive)>;

    // max_requests: PRN capacity of one grid (the channels of a receiver)
    AcquisitionService(const Acq_Conf& conf, uint32_t max_requests, int device = 0);
    ~AcquisitionService();
    AcquisitionService(const AcquisitionService&) = delete;
    AcquisitionService& operator=(const AcquisitionService&) = delete;

    // A channel arms an acquisition of `prn` with its sampled replica
    // (consumed_samples items).  One pending request per channel; a new request
    // replaces the old one.  Answered after the next complete block.
    void request(uint32_t channel, uint32_t prn, const std::complex<float>* code, Callback done);
    void cancel(uint32_t channel);
    size_t pending() const;

    // Shared input stream (item_type items): returns the items consumed.  Blocks
    // without any pending request are skipped without a launch.
    int work(const void* in, int ninput_items);

    // Device-ring form (gsdr_stream): the stream is pushed into the
    // GPU's IQ ring once (by whoever ingests it); the service runs its grids in
    // place on the ring's blocks [cursor, head), block after block, with no host
    // copy of its own.  The first call sets the block grid's origin at `head`.
    int work_ring(gsdr_stream* ring, uint64_t head);

    float threshold() const { return d_threshold; }
    uint64_t sample_counter() const { return d_sample_counter; }
    uint64_t grids_run() const { return d_grids; }

private:
    struct Request
    {
        uint32_t channel;
        uint32_t prn;
        std::vector<std::complex<float>> code;
        Callback done;
    };
    // grid over the pending requests on the current block: host buffer or ring
    void run_grid(gsdr_stream* ring = nullptr, uint64_t first_sample = 0);

    Acq_Conf d_conf;
    uint32_t d_max;
    uint32_t d_consumed;
    size_t d_isz;
    gsdr_acq* d_engine{nullptr};
    float d_threshold{0.0F};
    std::vector<Request> d_requests;
    bool d_codes_dirty{true};
    std::vector<uint8_t> d_buffer;
    uint32_t d_fill{0};
    uint64_t d_sample_counter{0};
    uint64_t d_grids{0};
    bool d_ring_started{false};
    uint64_t d_ring_cursor{0};  // absolute sample index of the next block on the ring
    mutable std::mutex d_mu;
};

#endif
