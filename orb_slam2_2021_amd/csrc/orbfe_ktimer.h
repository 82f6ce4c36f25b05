// orbfe_ktimer.h -- process-wide device-execution timing of the library's kernel launches
// (orbfe_ktimer_select / _read / _reset in include/orbfe.h). Not part of the C ABI.
//
// A selected launch goes through hipExtLaunchKernelGGL with a start and a stop event bound to the
// kernel dispatch itself, so the elapsed time is the dispatch's own begin/end timestamps -- the
// same interval rocprofv3's kernel trace reports -- and not the distance between two marker
// packets, which also counts the queue's wait for the packets ahead of it. Unselected launches
// (and every launch while nothing is selected) are plain hipLaunchKernelGGL calls behind one
// relaxed atomic load.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <atomic>

namespace orbfe_kt {
extern std::atomic<int> g_on;
// true: launch with (*e0, *e1) bound and call end(); false: launch plainly
bool begin(const char* name, int* slot, hipEvent_t* e0, hipEvent_t* e1);
void end(int slot, hipEvent_t e0, hipEvent_t e1);
}  // namespace orbfe_kt

// ORBFE_LAUNCH(name, kernel, grid, block, lds, stream, kernel args...)
#define ORBFE_LAUNCH(name, kernel, grid, block, lds, stream, ...)                                  \
  do {                                                                                             \
    int _kt_slot = -1;                                                                             \
    hipEvent_t _kt_e0 = nullptr, _kt_e1 = nullptr;                                                 \
    if (orbfe_kt::g_on.load(std::memory_order_relaxed) &&                                          \
        orbfe_kt::begin(name, &_kt_slot, &_kt_e0, &_kt_e1)) {                                      \
      hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, _kt_e0, _kt_e1, 0, __VA_ARGS__);     \
      orbfe_kt::end(_kt_slot, _kt_e0, _kt_e1);                                                     \
    } else {                                                                                       \
      hipLaunchKernelGGL(kernel, grid, block, lds, stream, __VA_ARGS__);                           \
    }                                                                                              \
  } while (0)
