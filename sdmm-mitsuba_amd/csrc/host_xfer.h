// host_xfer.h -- host transfer and scratch helpers shared by the runtime's
// translation units (sdmm_api.cpp defines them).  The rules they implement
// are stated in sdmm_api.cpp ("Host transfer and scratch rules") and in
// DESIGN.md section 2 ("Concurrency").
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <mutex>

namespace sdmm_detail {

// A device block grown on demand; owned by one (device, stream) pool entry.
struct StreamScratch {
    char* p = nullptr;
    size_t cap = 0;
};

// The calling thread's pinned bounce buffer of at least `bytes`.  Its previous
// contents are dead: every user synchronises its stream before it returns.
hipError_t bounce_buf(size_t bytes, char** out);

// The scratch entry of (device, stream), returned locked: hold the lock until
// the stream has been synchronised after the last use of the block.
std::unique_lock<std::mutex> stream_scratch(int device, hipStream_t st, StreamScratch** out);

// Grow s to at least `bytes` (the caller holds its lock, the stream is idle).
hipError_t scratch_reserve(StreamScratch& s, size_t bytes);

// Free every pool entry (sdmm_release_cached_scratch).
void release_stream_scratch();

}  // namespace sdmm_detail
