// comm_wait.hpp -- bounded waits for the multi-GPU frame gather (capi.cpp), header-only so the
// deadline logic is unit-tested on the CPU (tests/test_comm_wait_cpu.py builds a driver of it
// with g++; no GPU, no RCCL).
//
// The communicator is created non-blocking (ncclConfig_t.blocking = 0): RCCL calls return at
// once, possibly with ncclInProgress, and the outcome is polled with ncclCommGetAsyncError. A
// peer that dies before its send would otherwise leave rank 0 blocked forever in the stream
// synchronize after the grouped receive. Every wait here has a deadline; when it passes, or the
// communicator reports an error, the caller aborts the communicator (ncclCommAbort) and returns
// VK_ERROR_DEVICE_LOST -- the reference's convention of errors bubbling up as VkResult
// (VulkanComputeRayTracing.cpp:20-35).
#pragma once

#include <chrono>
#include <cstdint>
#include <cstdlib>
#include <thread>

namespace vcrt {

// What one poll of a pending operation reports.
enum class PollState { kDone, kPending, kFailed };

enum class WaitResult { kDone, kFailed, kTimedOut };

// Default deadline of one wait (communicator set-up, or one frame's gather): 120 s, or
// VCRT_COMM_TIMEOUT_MS from the environment (> 0).
inline int64_t comm_timeout_ms() {
    if (const char* e = std::getenv("VCRT_COMM_TIMEOUT_MS")) {
        const long long v = std::atoll(e);
        if (v > 0) return static_cast<int64_t>(v);
    }
    return 120000;
}

// Deadline of one frame's gather. The caller has waited for its own render (without a deadline)
// before the gather starts, but rank 0's receive still covers its peers' renders, which finish
// at about the same time in a balanced frame yet may lag by a fraction of a long one. So the
// exchange gets the base deadline plus four times this rank's own frame time: a slow but alive
// peer (a large spp, 4K, a stats build) is not mistaken for a lost one.
inline int64_t gather_timeout_ms(int64_t base_ms, double frame_ms) {
    const double extra = frame_ms > 0.0 ? 4.0 * frame_ms : 0.0;
    return base_ms + static_cast<int64_t>(extra < 9.0e15 ? extra + 1.0 : 9.0e15);
}

// Polls `poll` (returns PollState) until it reports done or failed, or until `timeout_ms` have
// passed since the call: kDone, kFailed or kTimedOut. The first polls run back to back (a gather
// normally completes within a frame), then the wait backs off to sleeps of 20 us, and of 200 us
// after ~20 ms (a frame waits at most that long past the gather's completion). `now`
// returns milliseconds on a monotonic clock (injectable for tests).
template <typename Poll, typename Now>
WaitResult wait_with_deadline(Poll&& poll, int64_t timeout_ms, Now&& now) {
    const int64_t start = now();
    for (uint32_t spin = 0;; spin++) {
        const PollState s = poll();
        if (s == PollState::kDone) return WaitResult::kDone;
        if (s == PollState::kFailed) return WaitResult::kFailed;
        if (now() - start >= timeout_ms) return WaitResult::kTimedOut;
        if (spin >= 64) std::this_thread::sleep_for(std::chrono::microseconds(spin < 1024 ? 20 : 200));
    }
}

inline int64_t steady_ms() {
    return std::chrono::duration_cast<std::chrono::milliseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

template <typename Poll>
WaitResult wait_with_deadline(Poll&& poll, int64_t timeout_ms) {
    return wait_with_deadline(poll, timeout_ms, steady_ms);
}

}  // namespace vcrt
