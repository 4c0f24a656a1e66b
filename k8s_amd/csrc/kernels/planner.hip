// Chip geometry for the launch planners (common.h planner_cus): the CU count every grid-sizing rule in the kernels
// is written against, read from the device instead of assumed (MI355X: 256 CUs in 8 XCDs).
#include <stdlib.h>

#include <atomic>

#include "common.h"

namespace k8s_amd {

namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_override{-1};  // -1: not read from the environment yet; 0: none
std::atomic<int> g_device_cus[kMaxDevices];

int env_override() {
  int v = g_override.load(std::memory_order_relaxed);
  if (v >= 0) return v;
  const char* e = getenv("K8S_AMD_PLANNER_CUS");
  int n = e ? atoi(e) : 0;
  if (n < 0) n = 0;
  int expected = -1;
  g_override.compare_exchange_strong(expected, n);
  return g_override.load(std::memory_order_relaxed);
}
}  // namespace

int planner_cus() {
  const int o = env_override();
  if (o > 0) return o;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDevices) return 256;
  int n = g_device_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  g_device_cus[dev].store(n, std::memory_order_relaxed);
  return n;
}

void set_planner_cus(int n) {
  env_override();  // the environment is read first, so a later first use cannot overwrite this value
  g_override.store(n > 0 ? n : 0, std::memory_order_relaxed);
}

}  // namespace k8s_amd
