// launch_state.cpp — per-device launch state of the kernel files, thread-safe.
//
// The C-ABI promises that plans may be shared across threads and streams
// (include/fory_rowfmt.h) and the host path keeps one context per device, so
// a process can drive several GPUs from several host threads. Everything a
// launch caches about a device lives here behind one mutex, keyed by the
// device current on the calling thread:
//   - the 160 KiB dynamic-LDS attribute of every kernel (hipFuncSetAttribute),
//     set once per (kernel, device) before that kernel's first launch there;
//   - the CU count (hipGetDeviceProperties) per device;
//   - occupancy answers (hipOccupancyMaxActiveBlocksPerMultiprocessor) per
//     (kernel, device, threads, LDS bytes) — the tile kernels size their LDS
//     images and staging slots by querying many candidate sizes.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "kernels.h"

#include <map>
#include <mutex>
#include <set>
#include <tuple>
#include <utility>

namespace fory_amd {

namespace {

std::mutex g_mu;

int current_device() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  return dev;
}

std::set<std::pair<const void*, int>>& lds_done() {
  static std::set<std::pair<const void*, int>> s;
  return s;
}

std::map<int, int>& cus_cache() {
  static std::map<int, int> m;
  return m;
}

std::map<std::tuple<const void*, int, int, size_t>, int>& occ_cache() {
  static std::map<std::tuple<const void*, int, int, size_t>, int> m;
  return m;
}

}  // namespace

void ensure_lds_cap(const void* kernel) {
  const int dev = current_device();
  std::lock_guard<std::mutex> lock(g_mu);
  if (!lds_done().insert({kernel, dev}).second) return;
  hipFuncAttributes attr{};  // dynamic LDS up to 160 KiB less the kernel's static LDS
  const size_t stat = hipFuncGetAttributes(&attr, kernel) == hipSuccess ? attr.sharedSizeBytes : 0;
  (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(160 * 1024 - stat));
}

int num_cus() {
  const int dev = current_device();
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = cus_cache().find(dev);
  if (it != cus_cache().end()) return it->second;
  int cus = 0;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) cus = prop.multiProcessorCount;
  if (cus <= 0) cus = 256;
  cus_cache()[dev] = cus;
  return cus;
}

int occupancy(const void* kernel, int threads, size_t lds) {
  const int dev = current_device();
  const auto key = std::make_tuple(kernel, dev, threads, lds);
  {
    std::lock_guard<std::mutex> lock(g_mu);
    auto it = occ_cache().find(key);
    if (it != occ_cache().end()) return it->second;
  }
  // the attribute must be in place before the query (LDS above the 64 KiB default)
  ensure_lds_cap(kernel);
  int blocks = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks, kernel, threads, lds) != hipSuccess) blocks = 0;
  std::lock_guard<std::mutex> lock(g_mu);
  occ_cache()[key] = blocks;
  return blocks;
}

// The plan's launch knobs (kernels.h / plan.h: LaunchKnobs), from the environment
// at plan creation; never read on a launch path.
LaunchKnobs knobs_from_env() {
  auto num = [](const char* name, int32_t unset) -> int32_t {
    const char* e = std::getenv(name);
    return e ? (int32_t)std::atoi(e) : unset;
  };
  auto set = [](const char* name) -> int32_t { return std::getenv(name) ? 1 : 0; };
  LaunchKnobs k{};
  const char* t = std::getenv("FORY_ROWFMT_VARTILE");
  k.no_tiles = t && std::atoi(t) == 0;
  const char* f = std::getenv("FORY_ROWFMT_VARFLAT");
  k.no_flat = f && std::atoi(f) == 0;
  k.var_cap = num("FORY_ROWFMT_VARCAP", 0);
  k.var_fit = set("FORY_ROWFMT_VARFIT");
  k.var_stg = num("FORY_ROWFMT_VARSTG", 0);
  k.spill_cap = num("FORY_ROWFMT_SPILLCAP", 0);
  k.var_nw = num("FORY_ROWFMT_VARNW", 0);
  k.sizes_program = set("FORY_ROWFMT_SIZES_PROGRAM");
  k.idx_frames = num("FORY_ROWFMT_IDXFRAMES", 0);
  k.prof = num("FORY_ROWFMT_VARPROF", 0) != 0;
  k.diag = set("FORY_ROWFMT_VARDIAG");
  k.var_enc = num("FORY_ROWFMT_VARENC", 0);
  k.var_xcd = num("FORY_ROWFMT_VARXCD", 0);
  k.dec_regs = num("FORY_ROWFMT_DECREGS", 0);
  k.tree_col = num("FORY_ROWFMT_TREECOL", 1);
  return k;
}

// FORY_ROWFMT_HOST_VERIFY=1: a host-path context reads back every host-to-device piece and
// compares it with the caller's bytes (host.cpp, verify_pieces); read at context creation.
bool host_verify_from_env() {
  const char* e = std::getenv("FORY_ROWFMT_HOST_VERIFY");
  return e && std::atoi(e) != 0;
}

}  // namespace fory_amd
