// Consumer side of the device IQ ring (stream.cpp) for the acquisition and
// tracking translation units.
#pragma once

#include <hip/hip_runtime.h>

#include "gsdr.h"

namespace gsdr
{
int stream_item_type(const gsdr_stream* s);
// device pointer of items [first, first + n) (contiguous; checked against the ring)
int stream_view(gsdr_stream* s, uint64_t first, uint64_t n, const void** ptr);
// the longest contiguous span ending at the head: [*first, *first + *n)
int stream_span(gsdr_stream* s, uint64_t* first, uint64_t* n);
// make `consumer` wait for the pushes so far; record the consumer's reads
int stream_acquire(gsdr_stream* s, hipStream_t consumer);
int stream_release(gsdr_stream* s, hipStream_t consumer);
}  // namespace gsdr
