// orbfe_ktimer.hip -- the process-wide kernel timer behind ORBFE_LAUNCH (orbfe_ktimer.h) and
// the orbfe_ktimer_* entry points (include/orbfe.h). Host code only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/orbfe.h"
#include "orbfe_device.h"
#include "orbfe_ktimer.h"

namespace orbfe_kt {
std::atomic<int> g_on{0};

namespace {
struct Pending {
  int slot;
  hipEvent_t e0, e1;
};
struct State {
  std::mutex mu;
  bool all = false;
  std::vector<std::string> selected;  // kernel names (all == false)
  std::vector<std::string> names;     // slot -> kernel name, in first-timed order
  std::vector<double> ms;
  std::vector<long long> launches;
  std::deque<Pending> pending;
  std::vector<hipEvent_t> pool;
};
State& st() {
  static State* s = new State();  // never destroyed: handles may outlive static teardown
  return *s;
}

void retire(State& s, const Pending& p, bool sync) {
  if (sync) hipEventSynchronize(p.e1);
  float t = 0.f;
  if (hipEventElapsedTime(&t, p.e0, p.e1) == hipSuccess) {
    s.ms[p.slot] += t;
    s.launches[p.slot] += 1;
  }
  s.pool.push_back(p.e0);
  s.pool.push_back(p.e1);
}

// completed launches at the head of the queue (bounded memory over long timed runs)
void harvest(State& s) {
  while (!s.pending.empty()) {
    if (hipEventQuery(s.pending.front().e1) != hipSuccess) {
      // NotReady may be recorded as the thread's last error: clear that one (not a real error
      // an earlier launch left), or the library's next hipGetLastError check would fail
      if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();
      break;
    }
    retire(s, s.pending.front(), false);
    s.pending.pop_front();
  }
}

hipEvent_t take(State& s) {
  if (!s.pool.empty()) {
    hipEvent_t e = s.pool.back();
    s.pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  return hipEventCreate(&e) == hipSuccess ? e : nullptr;
}
}  // namespace

bool begin(const char* name, int* slot, hipEvent_t* e0, hipEvent_t* e1) {
  State& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  if (!s.all && std::find(s.selected.begin(), s.selected.end(), name) == s.selected.end()) return false;
  auto it = std::find(s.names.begin(), s.names.end(), name);
  int k = (int)(it - s.names.begin());
  if (it == s.names.end()) {
    s.names.emplace_back(name);
    s.ms.push_back(0.0);
    s.launches.push_back(0);
  }
  if (s.pending.size() >= 4096) harvest(s);
  *e0 = take(s);
  *e1 = take(s);
  if (!*e0 || !*e1) {
    if (*e0) s.pool.push_back(*e0);
    if (*e1) s.pool.push_back(*e1);
    return false;
  }
  *slot = k;
  return true;
}

void end(int slot, hipEvent_t e0, hipEvent_t e1) {
  State& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  s.pending.push_back(Pending{slot, e0, e1});
}
}  // namespace orbfe_kt

extern "C" int orbfe_ktimer_select(const char* names) {
  using namespace orbfe_kt;
  State& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  s.selected.clear();
  s.all = false;
  const std::string v = names ? names : "";
  if (v == "*") {
    s.all = true;
  } else {
    size_t a = 0;
    while (a <= v.size()) {
      size_t b = v.find(',', a);
      if (b == std::string::npos) b = v.size();
      if (b > a) s.selected.emplace_back(v.substr(a, b - a));
      a = b + 1;
    }
  }
  g_on.store(s.all || !s.selected.empty() ? 1 : 0, std::memory_order_relaxed);
  return ORBFE_OK;
}

extern "C" int orbfe_ktimer_read(char* names, int name_len, double* total_ms, long long* launches,
                                 int cap, int* n) {
  using namespace orbfe_kt;
  if (!n || cap < 0 || (names && name_len <= 0)) return ORBFE_ERR_ARG;
  State& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  for (const Pending& p : s.pending) retire(s, p, true);
  s.pending.clear();
  *n = (int)s.names.size();
  for (int k = 0; k < (int)s.names.size() && k < cap; k++) {
    if (names) {
      std::strncpy(names + (size_t)k * name_len, s.names[k].c_str(), name_len - 1);
      names[(size_t)k * name_len + name_len - 1] = 0;
    }
    if (total_ms) total_ms[k] = s.ms[k];
    if (launches) launches[k] = s.launches[k];
  }
  return (int)s.names.size() > cap ? ORBFE_ERR_CAPACITY : ORBFE_OK;
}

// An empty one-workgroup kernel: the event interval it reports is the timer's own per-dispatch
// overhead (the marker and dispatch latency the dispatch-bound events include beyond the kernel's
// execution, which rocprofv3's kernel trace does not count).
__global__ void k_ktimer_nop() {}

extern "C" int orbfe_ktimer_calibrate(int device, int n, double* overhead_us) {
  if (!overhead_us || n <= 0) return ORBFE_ERR_ARG;
  ORBFE_HIP_CHECK(hipSetDevice(device));
  hipStream_t s = nullptr;
  ORBFE_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::vector<float> t;
  hipError_t err = hipEventCreate(&e0);
  if (err == hipSuccess) err = hipEventCreate(&e1);
  for (int i = 0; err == hipSuccess && i <= n; i++) {
    hipExtLaunchKernelGGL(k_ktimer_nop, dim3(1), dim3(64), 0, s, e0, e1, 0);
    err = hipEventSynchronize(e1);
    float ms = 0.f;
    if (err == hipSuccess) err = hipEventElapsedTime(&ms, e0, e1);
    if (err == hipSuccess && i > 0) t.push_back(ms);  // (the first launch loads the code object)
  }
  if (e0) hipEventDestroy(e0);
  if (e1) hipEventDestroy(e1);
  hipStreamDestroy(s);
  ORBFE_HIP_CHECK(err);
  std::sort(t.begin(), t.end());
  *overhead_us = 1e3 * (double)t[t.size() / 2];  // median
  return ORBFE_OK;
}

extern "C" int orbfe_ktimer_reset(void) {
  using namespace orbfe_kt;
  State& s = st();
  std::lock_guard<std::mutex> lk(s.mu);
  for (const Pending& p : s.pending) retire(s, p, true);
  s.pending.clear();
  std::fill(s.ms.begin(), s.ms.end(), 0.0);
  std::fill(s.launches.begin(), s.launches.end(), 0);
  return ORBFE_OK;
}
