// fc2_cpuacct.h -- CPU time per stage of the native read loop, for FC2_CALLER_TIMING: a stage adds
// its threads' CPU time (CLOCK_THREAD_CPUTIME_ID) around its work, so time a thread spends blocked
// counts nowhere.  fc2_caller_close prints the totals.
#pragma once
#include <stdint.h>
#include <stdlib.h>
#include <time.h>

#include <atomic>

namespace fc2 {
namespace cpu {

enum Stage { INFLATE, SPLIT, PARSE, CONSUME, NEXT_POOL, SUBMIT_POOL, SUBMIT_SERIAL, GZIP, kStages };

inline std::atomic<int64_t> *totals() {
    static std::atomic<int64_t> ns[kStages];
    return ns;
}

inline bool enabled() {
    static const bool on = getenv("FC2_CALLER_TIMING") != nullptr;
    return on;
}

inline int64_t thread_ns() {
    timespec t;
    clock_gettime(CLOCK_THREAD_CPUTIME_ID, &t);
    return (int64_t)t.tv_sec * 1000000000LL + t.tv_nsec;
}

class Scope {
  public:
    explicit Scope(Stage s) : s_(s), on_(enabled()), t0_(on_ ? thread_ns() : 0) {}
    ~Scope() {
        if (on_) totals()[s_] += thread_ns() - t0_;
    }
    Scope(const Scope &) = delete;
    Scope &operator=(const Scope &) = delete;

  private:
    Stage s_;
    bool on_;
    int64_t t0_;
};

}  // namespace cpu
}  // namespace fc2
