// Per-device launcher state of libstgcn_amd.so (SURVEY §8(b) threading: callers may drive several
// devices from several host threads, e.g. the reference's nn.DataParallel replicas).  Everything a
// launcher needs about the device comes from the device of the stream it launches on: its CU count
// (the persistent kernels' grid size) and the one-time MaxDynamicSharedMemorySize attribute of each
// kernel, both cached per device and safe under concurrent calls.
#include <hip/hip_runtime.h>

#include <atomic>
#include <map>
#include <mutex>
#include <utility>

#include "common.h"

namespace {
constexpr int kMaxDevices = 64;
std::atomic<int> g_cu_count[kMaxDevices];  // 0 = not queried yet (static storage: zero-initialised)
std::mutex g_attr_mu;
std::map<std::pair<const void*, int>, int> g_lds_attr;  // (kernel, device) -> dynamic LDS bytes allowed

int stream_device(hipStream_t s) {
  int dev = 0;
  if (s == nullptr || hipStreamGetDevice(s, &dev) != hipSuccess) (void)hipGetDevice(&dev);
  return dev;
}
}  // namespace

int stgcn_cu_count(hipStream_t s) {
  const int dev = stream_device(s);
  if (dev < 0 || dev >= kMaxDevices) return 256;
  int n = g_cu_count[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  g_cu_count[dev].store(n, std::memory_order_relaxed);
  return n;
}

int stgcn_lds_attr(const void* kernel, int bytes, hipStream_t s) {
  const int dev = stream_device(s);
  std::lock_guard<std::mutex> lock(g_attr_mu);
  int& have = g_lds_attr[{kernel, dev}];
  if (have >= bytes) return STGCN_OK;
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != dev) (void)hipSetDevice(dev);
  const hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  if (cur != dev) (void)hipSetDevice(cur);
  if (e != hipSuccess) return STGCN_EHIP;
  have = bytes;
  return STGCN_OK;
}
