// kcommon.h — device helpers and launch state shared by the kernel files
// (fixed.hip, scan.hip, varlen.hip, frames.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "kernels.h"

namespace fory_amd {

// ---------------------------------------------------------------------------
// Launch state (launch_state.cpp). Thread-safe and per device: a process may
// drive several GPUs from several host threads (one JNI context per device).
// ---------------------------------------------------------------------------
// hipFuncSetAttribute(MaxDynamicSharedMemorySize = 160 KiB) once per
// (kernel, current device), before the kernel's first launch there.
void ensure_lds_cap(const void* kernel);
// Compute units of the current device (cached per device).
int num_cus();
// hipOccupancyMaxActiveBlocksPerMultiprocessor, cached per (kernel, device,
// threads, LDS bytes); 0 on error.
int occupancy(const void* kernel, int threads, size_t lds);

namespace {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // native 16-B vector (SROA-friendly)

constexpr int kWG = 256;         // 4 waves
constexpr int kWaves = kWG / 64;

__device__ __forceinline__ void st32(uint8_t* p, uint32_t v) { *reinterpret_cast<uint32_t*>(p) = v; }
__device__ __forceinline__ uint32_t ld32(const uint8_t* p) { return *reinterpret_cast<const uint32_t*>(p); }

// Pointers read from a descriptor table are generic (flat) to the compiler;
// a flat access forces s_waitcnt vmcnt(0) lgkmcnt(0) before any dependent
// use. Cast them to the global address space so loads/stores are global_*.
#define GAS __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const GAS T* gp(const T* p) { return (const GAS T*)p; }
template <typename T>
__device__ __forceinline__ GAS T* gp(T* p) { return (GAS T*)p; }
// Bit updates of global words (no-return atomics on the global pointer: a generic one is a
// flat atomic, which makes every later wait a full vmcnt(0) + lgkmcnt(0) drain).
__device__ __forceinline__ void g_or(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_or(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void g_and(uint32_t* p, uint32_t v) {
  __hip_atomic_fetch_and(gp(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Loads the `width` low bytes of element `i` (little-endian, zero-extended).
__device__ __forceinline__ uint64_t load_elem(const uint8_t* base, int width, int64_t i) {
  switch (width) {
    case 8: return *gp(reinterpret_cast<const uint64_t*>(base + i * 8));
    case 4: return *gp(reinterpret_cast<const uint32_t*>(base + i * 4));
    case 2: return *gp(reinterpret_cast<const uint16_t*>(base + i * 2));
    default: return *gp(base + i);
  }
}

__device__ __forceinline__ void store_elem(uint8_t* base, int width, int64_t i, uint64_t v) {
  switch (width) {
    case 8: *gp(reinterpret_cast<uint64_t*>(base + i * 8)) = v; break;
    case 4: *gp(reinterpret_cast<uint32_t*>(base + i * 4)) = (uint32_t)v; break;
    case 2: *gp(reinterpret_cast<uint16_t*>(base + i * 2)) = (uint16_t)v; break;
    default: *gp(base + i) = (uint8_t)v; break;
  }
}

__device__ __forceinline__ uint8_t load_byte(const uint8_t* p) { return *gp(p); }
__device__ __forceinline__ void store_byte(uint8_t* p, uint8_t v) { *gp(p) = v; }

__device__ __forceinline__ void set_status(int32_t* status, int32_t code) {
  if (status) atomicCAS(status, 0, code);
}

template <int W>
__device__ __forceinline__ uint64_t ldw(const uint8_t* base, int64_t i) {
  if constexpr (W == 8) return *gp(reinterpret_cast<const uint64_t*>(base) + i);
  if constexpr (W == 4) return *gp(reinterpret_cast<const uint32_t*>(base) + i);
  if constexpr (W == 2) return *gp(reinterpret_cast<const uint16_t*>(base) + i);
  return *gp(base + i);
}

template <int W>
__device__ __forceinline__ void stw(uint8_t* base, int64_t i, uint64_t v) {
  if constexpr (W == 8) *gp(reinterpret_cast<uint64_t*>(base) + i) = v;
  else if constexpr (W == 4) *gp(reinterpret_cast<uint32_t*>(base) + i) = (uint32_t)v;
  else if constexpr (W == 2) *gp(reinterpret_cast<uint16_t*>(base) + i) = (uint16_t)v;
  else *gp(base + i) = (uint8_t)v;
}

template <typename K>
void raise_lds_cap(K* kernel) {
  ensure_lds_cap(reinterpret_cast<const void*>(kernel));
}

template <typename K>
int occupancy_of(K* kernel, int threads, size_t lds) {
  return occupancy(reinterpret_cast<const void*>(kernel), threads, lds);
}

// Persistent grid: resident workgroups per CU (occupancy query) x CUs.
template <typename K>
int64_t persistent_grid(K* kernel, size_t lds, int64_t tiles, int wg = kWG) {
  int per_cu = occupancy_of(kernel, wg, lds);
  if (per_cu <= 0) per_cu = 1;
  const int64_t g = (int64_t)per_cu * num_cus();
  return tiles < g ? tiles : g;
}

}  // namespace
}  // namespace fory_amd
