// pinned_probe — does a hipMemcpyAsync out of a pinned host block ever deliver bytes
// the host overwrote before the copy was queued? (the staged pageable
// host encode once delivered a whole chunk's f0 column and part of f1 wrong,
// profiles/r05/intermittent/.) Deterministic sequences, each on a block of one
// allocation kind and size, every byte checked:
//   d2h_h2d   DMA device(P1) -> block; sync; host writes P2 into the block; DMA block ->
//             device; sync; is the device P2?  (the staging ring: a block that last took a
//             D2H piece is next filled by the host for an H2D piece)
//   d2h_h2d_x the same with the D2H on one stream + hipEventSynchronize and the H2D on
//             another (host.cpp: rows leave on s_out, columns arrive on s_in)
//   h2d_h2d   host P1 -> block -> device; host P2 -> block -> device; second copy P2?
//   realloc   DMA device(P1) -> block; hipHostFree; hipHostMalloc (same kind and size:
//             often the same address); host writes P2; DMA -> device; P2?  (a context's
//             blocks are freed and the next context's blocks take the same pages)
//   kernel    a kernel reads the block through its device mapping after a D2H and a
//             host overwrite (what a blit copy kernel does)
// Host writes use the host path's own non-temporal copy (stream_copy) or memcpy.
// Kinds: nc = hipHostMallocPortable (round 5's staging before c093321), coh =
// Portable | Coherent (the staging now), ncx = Portable | NonCoherent, reg = malloc +
// hipHostRegister. Output: one JSON line per (kind, size, sequence, writer): bytes
// checked, bytes wrong, wrong bytes equal to the stale pattern.
// Also: hipHostRegister + hipHostUnregister throughput of touched pageable memory
// (VERDICT r5 item 7 asks for per-call registration of pageable column interiors).
#include <hip/hip_runtime.h>
#include <emmintrin.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__host__ __device__ inline uint8_t pat(uint32_t seed, uint64_t i) {
  uint32_t x = (uint32_t)i * 2654435761u + seed * 40503u + (uint32_t)(i >> 12);
  x ^= x >> 13;
  return (uint8_t)(x * 97u + seed);
}

__global__ void fill_kernel(uint8_t* d, uint64_t n, uint32_t seed) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    d[i] = pat(seed, i);
}

__global__ void read_kernel(const uint8_t* h, uint8_t* d, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    d[i] = h[i];
}

static void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
  const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
  std::memcpy(dst, src, head < n ? head : n);
  size_t i = head;
  for (; i + 64 <= n; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  if (i < n) std::memcpy(dst + i, src + i, n - i);
  _mm_sfence();
}

struct Block {
  uint8_t* p = nullptr;
  int kind = 0;
  size_t n = 0;
};

static const char* kind_name(int k) { return k == 0 ? "nc" : k == 1 ? "coh" : k == 2 ? "ncx" : "reg"; }

static Block alloc_block(int kind, size_t n) {
  Block b;
  b.kind = kind;
  b.n = n;
  if (kind == 3) {
    void* p = nullptr;
    if (posix_memalign(&p, 4096, n)) exit(1);
    memset(p, 0, n);
    CK(hipHostRegister(p, n, hipHostRegisterDefault));
    b.p = static_cast<uint8_t*>(p);
  } else {
    const unsigned fl = kind == 0 ? hipHostMallocPortable
                        : kind == 1 ? (hipHostMallocPortable | hipHostMallocCoherent)
                                    : (hipHostMallocPortable | hipHostMallocNonCoherent);
    CK(hipHostMalloc(reinterpret_cast<void**>(&b.p), n, fl));
  }
  return b;
}

static void free_block(Block& b) {
  if (!b.p) return;
  if (b.kind == 3) {
    CK(hipHostUnregister(b.p));
    free(b.p);
  } else {
    CK(hipHostFree(b.p));
  }
  b.p = nullptr;
}

struct Result {
  uint64_t checked = 0, wrong = 0, stale = 0;
  int same_addr = 0;
};

static void host_write(uint8_t* blk, const uint8_t* src, size_t n, bool nt) {
  if (nt && n >= 64) stream_copy(blk, src, n);
  else memcpy(blk, src, n);
}

static void check(const uint8_t* got, size_t n, uint32_t want, uint32_t old, Result& r) {
  for (size_t i = 0; i < n; ++i) {
    const uint8_t w = pat(want, i);
    ++r.checked;
    if (got[i] != w) {
      ++r.wrong;
      if (got[i] == pat(old, i)) ++r.stale;
    }
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 8;
  const size_t sizes[] = {4096, 32768, 65536, 262144, 1 << 20, 16 << 20};
  CK(hipSetDevice(0));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  const size_t maxn = 16 << 20;
  uint8_t *dA, *dB;
  CK(hipMalloc(&dA, maxn));
  CK(hipMalloc(&dB, maxn));
  std::vector<uint8_t> src(maxn), got(maxn);
  const char* seqs[] = {"d2h_h2d", "d2h_h2d_x", "h2d_h2d", "realloc", "kernel"};
  uint32_t seed = 1;
  for (int kind = 0; kind < 4; ++kind)
    for (size_t n : sizes)
      for (int sq = 0; sq < 5; ++sq)
        for (int nt = 0; nt < 2; ++nt) {
          if (kind == 3 && sq == 3) continue;  // realloc of a registration: malloc'd pages
          Result r;
          Block b = alloc_block(kind, n);
          for (int it = 0; it < iters; ++it) {
            const uint32_t p1 = seed++, p2 = seed++;
            for (size_t i = 0; i < n; ++i) src[i] = pat(p2, i);
            if (sq == 2) {  // h2d_h2d: P1 through the block first
              std::vector<uint8_t> s1v(n);
              for (size_t i = 0; i < n; ++i) s1v[i] = pat(p1, i);
              host_write(b.p, s1v.data(), n, nt);
              CK(hipMemcpyAsync(dB, b.p, n, hipMemcpyHostToDevice, s1));
              CK(hipStreamSynchronize(s1));
            } else {  // device P1 -> block
              hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, s1, dA, (uint64_t)n, p1);
              CK(hipMemcpyAsync(b.p, dA, n, hipMemcpyDeviceToHost, s1));
              if (sq == 1) {
                CK(hipEventRecord(ev, s1));
                CK(hipEventSynchronize(ev));
              } else {
                CK(hipStreamSynchronize(s1));
              }
            }
            if (sq == 3) {
              uint8_t* before = b.p;
              free_block(b);
              b = alloc_block(kind, n);
              r.same_addr += b.p == before;
            }
            host_write(b.p, src.data(), n, nt);
            hipStream_t sh = sq == 1 ? s2 : s1;
            if (sq == 4) {
              void* dp = nullptr;
              CK(hipHostGetDevicePointer(&dp, b.p, 0));
              hipLaunchKernelGGL(read_kernel, dim3(256), dim3(256), 0, sh, static_cast<const uint8_t*>(dp), dB,
                                 (uint64_t)n);
            } else {
              CK(hipMemcpyAsync(dB, b.p, n, hipMemcpyHostToDevice, sh));
            }
            CK(hipStreamSynchronize(sh));
            CK(hipMemcpy(got.data(), dB, n, hipMemcpyDeviceToHost));
            check(got.data(), n, p2, p1, r);
          }
          free_block(b);
          printf("{\"kind\": \"%s\", \"bytes\": %zu, \"seq\": \"%s\", \"writer\": \"%s\", \"iters\": %d, "
                 "\"checked\": %llu, \"wrong\": %llu, \"stale\": %llu, \"same_addr\": %d}\n",
                 kind_name(kind), n, seqs[sq], nt ? "nt" : "memcpy", iters, (unsigned long long)r.checked,
                 (unsigned long long)r.wrong, (unsigned long long)r.stale, r.same_addr);
          fflush(stdout);
        }
  // registration cost of touched pageable memory
  for (size_t mb : {64, 256, 1024}) {
    const size_t n = mb << 20;
    void* p = nullptr;
    if (posix_memalign(&p, 4096, n)) return 1;
    memset(p, 1, n);
    double reg = 1e30, unreg = 1e30;
    for (int it = 0; it < 3; ++it) {
      auto t0 = std::chrono::steady_clock::now();
      CK(hipHostRegister(p, n, hipHostRegisterDefault));
      auto t1 = std::chrono::steady_clock::now();
      CK(hipHostUnregister(p));
      auto t2 = std::chrono::steady_clock::now();
      reg = std::min(reg, std::chrono::duration<double>(t1 - t0).count());
      unreg = std::min(unreg, std::chrono::duration<double>(t2 - t1).count());
    }
    printf("{\"register_mib\": %zu, \"register_ms\": %.3f, \"unregister_ms\": %.3f, \"register_gbs\": %.2f, "
           "\"register_plus_unregister_gbs\": %.2f}\n",
           mb, reg * 1e3, unreg * 1e3, n / reg / 1e9, n / (reg + unreg) / 1e9);
    fflush(stdout);
    free(p);
  }
  return 0;
}
