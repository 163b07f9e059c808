// One GPU acquisition grid serving every channel's acquisition requests
// (SURVEY.md §8f rank 2).
//
// In the reference every channel owns a pcps_acquisition block that searches one
// PRN per call over the shared sample stream (GNSSFlowgraph::connect wires the
// same signal-conditioner output to all acquisition blocks,
// src/core/receiver/gnss_flowgraph.cc:1796-1901; the channel FSM arms one
// acquisition per channel, src/algorithms/channel/libs/channel_fsm.cc:80-135).
// Here the channels post requests (PRN + replica + decision callback) to one
// service, which answers every armed request on each complete block of
// consumed_samples items with one batched acquisition_core over the armed PRNs
// (the positive/negative event of pcps_acquisition::acquisition_core, :781-829,
// single dwell).
//
// Code spectra stay resident per request slot: a channel's request uploads and
// transforms its replica only when the slot's PRN changes (set_local_code runs once
// per PRN assignment in the reference, pcps_acquisition.cc:176-209); re-arming the
// same PRN after an answer costs nothing.  On the device ring the service runs up
// to batch_blocks ready blocks per launch with up to two launches in flight (the
// second queued behind the first, so the GPU does not idle while the host answers
// the first); a launch's results are collected before a third is submitted or at
// flush().  A request stays armed until its answer is processed, so a launch
// submitted before that searches it again; a request re-armed by its callback with
// the same PRN is answered by the next block of the launches in flight.
#ifndef GSDR_HOST_ACQUISITION_SERVICE_H
#define GSDR_HOST_ACQUISITION_SERVICE_H

#include <complex>
#include <cstdint>
#include <deque>
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

    // max_requests: PRN slots of one grid (the channels of a receiver);
    // batch_blocks: blocks per launch on the device ring
    AcquisitionService(const Acq_Conf& conf, uint32_t max_requests, int device = 0, uint32_t batch_blocks = 4);
    ~AcquisitionService();
    AcquisitionService(const AcquisitionService&) = delete;
    AcquisitionService& operator=(const AcquisitionService&) = delete;

    // A channel arms an acquisition of `prn` with its sampled replica
    // (consumed_samples items, read now only if the channel's slot does not hold
    // this PRN's spectrum yet).  One pending request per channel; a new request
    // replaces the old one.  Answered on a later complete block.  May be called
    // from a callback.
    void request(uint32_t channel, uint32_t prn, const std::complex<float>* code, Callback done);
    void cancel(uint32_t channel);
    size_t pending() const;

    // Shared input stream (item_type items): returns the items consumed.  Each
    // complete block with any armed request is one synchronous grid.
    int work(const void* in, int ninput_items);

    // Device-ring form (gsdr_stream): the stream is pushed into the
    // GPU's IQ ring once (by whoever ingests it); the service runs its grids in
    // place on the ring's blocks [cursor, head), batch_blocks per launch, and
    // answers the launch in flight at the next call.  The first call sets the block
    // grid's origin at `head`.  Returns the blocks consumed.
    int work_ring(gsdr_stream* ring, uint64_t head);
    // answers the launches in flight (if any)
    void flush();

    float threshold() const { return d_threshold; }
    uint64_t sample_counter() const { return d_sample_counter; }
    uint64_t grids_run() const { return d_grids; }          // blocks searched
    uint64_t launches() const { return d_launches; }        // grid launches
    uint64_t code_uploads() const { return d_code_uploads; }  // set_local_code calls

private:
    struct Slot
    {
        bool used{false};    // holds a channel's request slot
        uint32_t channel{0};
        uint32_t prn{0};
        bool loaded{false};  // the engine's spectrum of this slot is prn's
        uint64_t gen{0};     // spectrum generation (bumped by each upload)
        bool armed{false};
        Callback done;
        std::vector<std::complex<float>> code;  // replica waiting for upload (!loaded)
    };
    struct Flight
    {
        uint32_t nblocks{0};
        std::vector<uint64_t> gen;  // per slot at submission (slots [0, nprn))
    };
    static constexpr size_t kMaxFlights = 2;  // gsdr_acq_submit_stream's queue depth
    void collect_oldest();
    // uploads the armed slots' pending replicas and sets the active PRN count;
    // false when nothing is armed (lock held)
    bool prepare_locked(std::vector<uint64_t>& gen);
    // answers block b of a result set (block-major, nprn per block); returns the
    // callbacks to run outside the lock
    void answer(const std::vector<gsdr_acq_result>& res, uint32_t nblocks, uint32_t nprn, const std::vector<uint64_t>& gen,
        bool device_error);

    Acq_Conf d_conf;
    uint32_t d_max;
    uint32_t d_consumed;
    size_t d_isz;
    uint32_t d_batch;
    gsdr_acq* d_engine{nullptr};
    float d_threshold{0.0F};
    std::vector<Slot> d_slots;
    std::vector<uint8_t> d_buffer;
    uint32_t d_fill{0};
    uint64_t d_sample_counter{0};
    uint64_t d_grids{0};
    uint64_t d_launches{0};
    uint64_t d_code_uploads{0};
    bool d_ring_started{false};
    uint64_t d_ring_cursor{0};  // absolute sample index of the next block on the ring
    std::deque<Flight> d_flights;  // launches in flight, oldest first
    std::vector<gsdr_acq_result> d_res;
    mutable std::mutex d_mu;
};

#endif
