// Consumer side of the device IQ ring (stream.cpp) for the acquisition and
// tracking translation units.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

#include "gsdr.h"

namespace gsdr
{
int stream_item_type(const gsdr_stream* s);
int stream_device(const gsdr_stream* s);

// A consumer launch reads the ring under one hold of the ring's lock, from
// choosing its window to recording its reader event, so a push from another
// thread (the GNU Radio producer) cannot land between the two and overwrite the
// window the kernel is about to read: the push waits for the lock, then its copy
// waits for the recorded reader event.
class StreamReader
{
public:
    explicit StreamReader(gsdr_stream* s);
    StreamReader(const StreamReader&) = delete;
    StreamReader& operator=(const StreamReader&) = delete;
    // device pointer of items [first, first + n) (contiguous; checked against the ring)
    int view(uint64_t first, uint64_t n, const void** ptr);
    // the longest contiguous span ending at the head: [*first, *first + *n)
    int span(uint64_t* first, uint64_t* n);
    // make `consumer` wait for the pushes so far
    int acquire(hipStream_t consumer);
    // record the consumer's reads (a push overwriting the oldest item viewed waits for them)
    int release(hipStream_t consumer);

private:
    gsdr_stream* s_;
    uint64_t lo_{UINT64_MAX};  // the oldest item viewed
    std::unique_lock<std::mutex> lk_;
};
}  // namespace gsdr
