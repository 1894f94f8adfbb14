// respool.h -- process-wide caches of the HIP resources the drop-in objects
// (OLAAccumulator, FrameQueue, FFT plans) create per instance: non-blocking
// streams, pinned host blocks, and device memory from the stream-ordered
// allocator with its release threshold raised.  The reference constructs these
// objects inside its benchmark loops (bench/performance_benchmark.cc:181-210);
// a stream, a pinned block or a hipFree per construction costs more than the
// object's whole per-frame work.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>

namespace crlot {

// A non-blocking stream of `device` (created on first use, reused after put).
hipError_t pool_stream(int device, hipStream_t* out);
void pool_stream_put(int device, hipStream_t s);

// A timing-disabled event of `device` (created on first use, reused after put).
hipError_t pool_event(int device, hipEvent_t* out);
void pool_event_put(int device, hipEvent_t ev);

// A pinned host block of at least `bytes` (*cap: its size; power-of-two classes).
hipError_t pool_pinned(size_t bytes, void** out, size_t* cap);
void pool_pinned_put(void* p, size_t cap);

// Device memory, stream-ordered on s (hipMallocAsync / hipFreeAsync on the
// device's default pool, whose release threshold is raised on first use so
// freed blocks stay cached instead of being unmapped at every synchronisation).
hipError_t pool_malloc(int device, void** out, size_t bytes, hipStream_t s);
void pool_free(void* p, hipStream_t s);

}  // namespace crlot
