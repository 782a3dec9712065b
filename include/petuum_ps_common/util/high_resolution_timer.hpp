// high_resolution_timer.hpp — HighResolutionTimer (src/petuum_ps_common/util/high_resolution_timer.hpp):
// seconds since construction or restart().
#pragma once
#include <chrono>

namespace petuum {

class HighResolutionTimer {
 public:
  HighResolutionTimer() { restart(); }
  void restart() { start_ = std::chrono::steady_clock::now(); }
  double elapsed() const {
    return std::chrono::duration<double>(std::chrono::steady_clock::now() - start_).count();
  }
  double elapsed_max() const { return 1e18; }
  double elapsed_min() const { return 1e-9; }

 private:
  std::chrono::steady_clock::time_point start_;
};

}  // namespace petuum
