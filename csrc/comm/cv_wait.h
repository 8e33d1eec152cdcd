// Timed condition-variable waits on steady-clock deadlines.
//
// Under ThreadSanitizer (DMLC_TSAN) the wait is made on the equivalent
// system-clock deadline instead: libstdc++ 11 implements a steady-clock
// wait_until with pthread_cond_clockwait, which GCC 11's ThreadSanitizer does
// not intercept, so every such wait would show up as a false double lock and
// a stream of false races on the data the mutex guards. The system-clock form
// goes through pthread_cond_timedwait, which it does intercept.
#pragma once
#include <chrono>
#include <condition_variable>
#include <mutex>

namespace dmlc {

inline std::cv_status cv_wait_until(std::condition_variable& cv, std::unique_lock<std::mutex>& g,
                                    std::chrono::steady_clock::time_point deadline) {
#ifdef DMLC_TSAN
  const auto left = deadline - std::chrono::steady_clock::now();
  const auto st = cv.wait_until(g, std::chrono::system_clock::now() +
                                       std::chrono::duration_cast<std::chrono::system_clock::duration>(left));
  (void)st;
  return std::chrono::steady_clock::now() >= deadline ? std::cv_status::timeout : std::cv_status::no_timeout;
#else
  return cv.wait_until(g, deadline);
#endif
}

}  // namespace dmlc
