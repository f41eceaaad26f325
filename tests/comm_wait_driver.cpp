// Unit driver of vulkancomputeraytracing_amd/csrc/comm_wait.hpp (the deadline logic of the
// multi-GPU gather), built and run on the CPU by tests/test_comm_wait_cpu.py. Prints one line
// per case: "<name> <result> <polls> <elapsed ms>".
#include <cstdio>
#include <cstdlib>

#include "comm_wait.hpp"

using vcrt::PollState;
using vcrt::WaitResult;

static const char* name(WaitResult r) {
    return r == WaitResult::kDone ? "done" : r == WaitResult::kFailed ? "failed" : "timeout";
}

int main() {
    // a fake clock: every call advances 1 ms
    int64_t fake = 0;
    auto tick = [&fake] { return fake++; };

    // done on the 5th poll, well before the deadline
    int polls = 0;
    WaitResult r = vcrt::wait_with_deadline(
        [&] { return ++polls < 5 ? PollState::kPending : PollState::kDone; }, 1000, tick);
    std::printf("done_after_5 %s %d\n", name(r), polls);

    // an asynchronous error on the 3rd poll
    polls = 0;
    fake = 0;
    r = vcrt::wait_with_deadline(
        [&] { return ++polls < 3 ? PollState::kPending : PollState::kFailed; }, 1000, tick);
    std::printf("failed_after_3 %s %d\n", name(r), polls);

    // never completes: times out once the fake clock passes 50 ms (and not before)
    polls = 0;
    fake = 0;
    r = vcrt::wait_with_deadline([&] { ++polls; return PollState::kPending; }, 50, tick);
    std::printf("pending_forever %s %d %lld\n", name(r), polls, static_cast<long long>(fake));

    // completes on the 50th poll, the one at which the deadline would pass: done wins
    polls = 0;
    fake = 0;
    r = vcrt::wait_with_deadline(
        [&] { return ++polls < 50 ? PollState::kPending : PollState::kDone; }, 50, tick);
    std::printf("done_at_deadline %s %d\n", name(r), polls);

    // the real clock: a 200 ms deadline on an operation that never completes
    const int64_t t0 = vcrt::steady_ms();
    polls = 0;
    r = vcrt::wait_with_deadline([&] { ++polls; return PollState::kPending; }, 200);
    const int64_t dt = vcrt::steady_ms() - t0;
    std::printf("real_clock %s %d %lld\n", name(r), polls, static_cast<long long>(dt));

    // a slow but alive peer: base deadline 50 ms, this rank's frame 30 ms -> 50 + 121 ms; the
    // gather completes at 150 ms (past the base deadline alone) and is done, not lost
    polls = 0;
    fake = 0;
    const int64_t gt = vcrt::gather_timeout_ms(50, 30.0);
    r = vcrt::wait_with_deadline(
        [&] { return ++polls < 150 ? PollState::kPending : PollState::kDone; }, gt, tick);
    std::printf("slow_peer %s %d %lld\n", name(r), polls, static_cast<long long>(gt));
    // ... and a peer that never sends still times out at that deadline
    polls = 0;
    fake = 0;
    r = vcrt::wait_with_deadline([&] { ++polls; return PollState::kPending; }, gt, tick);
    std::printf("lost_peer %s %d\n", name(r), polls);
    std::printf("gather_ms %lld %lld\n", static_cast<long long>(vcrt::gather_timeout_ms(120000, 0.0)),
                static_cast<long long>(vcrt::gather_timeout_ms(120000, 2670.5)));

    // the environment override of the default deadline
    std::printf("default_ms %lld\n", static_cast<long long>(vcrt::comm_timeout_ms()));
    return 0;
}
