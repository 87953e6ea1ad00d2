// wait_test.cpp — mtcp_amd/csrc/wait.hpp on the CPU (no GPU, no HIP calls:
// the polls are driven by fake queries).  Built with g++ and run by
// tests/test_wait_rules.py; prints one JSON line.
#include <stdio.h>

#include <chrono>

#include "../../mtcp_amd/csrc/wait.hpp"

using mtcp_wait::Deadline;
using mtcp_wait::poll;

int main() {
    // ready after 100 polls, no bound: OK after exactly 100 queries
    int n1 = 0;
    const int rc1 = poll([&] { return ++n1 < 100 ? hipErrorNotReady : hipSuccess; }, Deadline(0));
    // never ready, 20 ms bound: ETIMEDOUT, not before the deadline, soon after
    int n2 = 0;
    const auto t0 = std::chrono::steady_clock::now();
    const int rc2 = poll([&] { ++n2; return hipErrorNotReady; }, Deadline(20000));
    const double ms2 = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    // a runtime error: EIO at once
    int n3 = 0;
    const int rc3 = poll([&] { ++n3; return hipErrorInvalidValue; }, Deadline(20000));
    // the deadline already passed but the work is done: the result wins
    Deadline past(1);
    while (!past.passed()) {
    }
    int n4 = 0;
    const int rc4 = poll([&] { ++n4; return hipSuccess; }, past);
    // an unbounded deadline never passes
    const Deadline none(0);
    printf("{\"ready_after_100\": [%d, %d], \"never_ready_20ms\": [%d, %d, %.2f], \"error\": [%d, %d], "
           "\"done_after_deadline\": [%d, %d], \"unbounded\": [%d, %d]}\n",
           rc1, n1, rc2, n2 > 1, ms2, rc3, n3, rc4, n4, (int)none.bounded, (int)none.passed());
    return 0;
}
