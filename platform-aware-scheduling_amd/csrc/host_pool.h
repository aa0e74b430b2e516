// host_pool.h — the host worker threads shared by the wire decoder and encoders.
//
// Defined in wire_decode.cpp (its WorkerPool: threads kept across calls, one parallel step at
// a time, fresh threads for a concurrent caller).  Host C++ only.
#pragma once

#include <cstdint>
#include <functional>

namespace pas {

// Threads for `bytes` of host work: one per MiB, at most pas_decode_set_threads' value (or
// min(hardware threads, 16) when it is 0), at least 1.
int host_threads_for(int64_t bytes);

// f(i) for i in [0, n) on the pool, on up to `threads` threads (0: n), each taking the next i
// until none is left; false (nothing run) when no thread can be started.
bool host_parallel(int n, const std::function<void(int)>& f, int threads = 0);

// Work pieces per thread of a parallel step: more pieces than threads balance a thread the
// host delays.
constexpr int kHostPieces = 4;

}  // namespace pas
