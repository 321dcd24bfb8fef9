// ring_probe — the host path's staging ring in isolation: does a
// pinned block get rewritten by the host before the DMA that last read it has read it?
// host.cpp's H2D protocol per piece: take block j = next++ % 8; if its last DMA's event
// is recorded, hipEventSynchronize it; memcpy the piece into the block; hipMemcpyAsync
// block -> device on the stream; hipEventRecord(ev[j]). One "context" = fresh streams,
// fresh events and fresh blocks (host.cpp: per fory_host_ctx), then one chunk of
// Struct104 at 8192 records: 104 column pieces of 32 / 64 KiB in schema order
// (f0 i32, f1 i64, f10 f32, f100 i32, ...), as in the failing
// test_host_pageable_pieces_over_a_mib[struct104-20011-8192]. After the stream drains,
// every device slice is compared with its source; a wrong slice reports which source
// column it equals (the piece that took its block next = an early block reuse).
// Variants: block kind (nc / coh), events and streams fresh per context or reused,
// sdma via HSA_ENABLE_SDMA in the environment.
// Usage: ring_probe <contexts> <kind: 0 nc, 1 coh> <fresh: 1 new streams+events per context>
#include <hip/hip_runtime.h>

#include <algorithm>
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

constexpr int kBlocks = 8;
constexpr size_t kBlock = size_t(16) << 20;

int main(int argc, char** argv) {
  const int contexts = argc > 1 ? atoi(argv[1]) : 100;
  const int kind = argc > 2 ? atoi(argv[2]) : 0;
  const int fresh = argc > 3 ? atoi(argv[3]) : 1;
  const int rows = 8192;
  // Struct104 schema order: names f0..f103 sorted as strings; f{4k}: int, f{4k+1}: long,
  // f{4k+2}: float, f{4k+3}: double
  std::vector<std::string> names;
  for (int i = 0; i < 104; ++i) names.push_back("f" + std::to_string(i));
  std::sort(names.begin(), names.end());
  std::vector<int> width;
  for (auto& s : names) width.push_back((atoi(s.c_str() + 1) % 2) ? 8 : 4);
  const int ncol = (int)width.size();
  std::vector<std::vector<uint8_t>> src(ncol);
  std::vector<size_t> off(ncol + 1, 0);
  for (int i = 0; i < ncol; ++i) {
    src[i].resize((size_t)rows * width[i]);
    for (size_t b = 0; b < src[i].size(); ++b) src[i][b] = (uint8_t)(b * 131 + i * 977 + (b >> 9) * 7 + 1);
    off[i + 1] = off[i] + ((src[i].size() + 255) & ~size_t(255));
  }
  CK(hipSetDevice(0));
  uint8_t* dev = nullptr;
  CK(hipMalloc(&dev, off[ncol]));
  std::vector<uint8_t> got(off[ncol]);
  hipStream_t s = nullptr;
  hipEvent_t ev[kBlocks] = {};
  long long bad_ctx = 0, bad_pieces = 0, early_reuse = 0;
  for (int ctx = 0; ctx < contexts; ++ctx) {
    if (fresh || !s) {
      if (s) CK(hipStreamDestroy(s));
      CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
      for (auto& e : ev) {
        if (e) CK(hipEventDestroy(e));
        e = nullptr;
      }
    }
    uint8_t* mem = nullptr;
    const unsigned fl = kind ? (hipHostMallocPortable | hipHostMallocCoherent) : hipHostMallocPortable;
    CK(hipHostMalloc(reinterpret_cast<void**>(&mem), kBlock * kBlocks, fl));
    for (auto& e : ev)
      if (!e) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    CK(hipMemset(dev, 0, off[ncol]));  // (the context's arena is zeroed synchronously at creation)
    bool inflight[kBlocks] = {};
    int next = 0;
    for (int i = 0; i < ncol; ++i) {
      const int j = next;
      next = (next + 1) % kBlocks;
      if (inflight[j]) CK(hipEventSynchronize(ev[j]));
      uint8_t* blk = mem + (size_t)j * kBlock;
      memcpy(blk, src[i].data(), src[i].size());
      CK(hipMemcpyAsync(dev + off[i], blk, src[i].size(), hipMemcpyHostToDevice, s));
      CK(hipEventRecord(ev[j], s));
      inflight[j] = true;
    }
    CK(hipStreamSynchronize(s));
    CK(hipMemcpy(got.data(), dev, off[ncol], hipMemcpyDeviceToHost));
    int nbad = 0;
    for (int i = 0; i < ncol; ++i) {
      if (!memcmp(got.data() + off[i], src[i].data(), src[i].size())) continue;
      ++nbad;
      size_t wrong = 0;
      for (size_t b = 0; b < src[i].size(); ++b) wrong += got[off[i] + b] != src[i][b];
      int equals = -1;  // a later piece of the same block?
      for (int q = i + kBlocks; q < ncol && equals < 0; q += kBlocks)
        if (src[q].size() >= 64 && !memcmp(got.data() + off[i], src[q].data(), 64)) equals = q;
      early_reuse += equals >= 0;
      printf("{\"ctx\": %d, \"piece\": %d, \"name\": \"%s\", \"bytes\": %zu, \"wrong\": %zu, \"starts_like_piece\": %d}\n",
             ctx, i, names[i].c_str(), src[i].size(), wrong, equals);
    }
    bad_pieces += nbad;
    bad_ctx += nbad > 0;
    CK(hipHostFree(mem));
    if (ctx % 50 == 49) {
      fprintf(stderr, "ctx %d bad_ctx %lld\n", ctx + 1, bad_ctx);
    }
  }
  printf("{\"summary\": true, \"contexts\": %d, \"kind\": \"%s\", \"fresh\": %d, \"bad_contexts\": %lld, "
         "\"bad_pieces\": %lld, \"early_reuse_pieces\": %lld}\n",
         contexts, kind ? "coh" : "nc", fresh, bad_ctx, bad_pieces, early_reuse);
  return 0;
}
