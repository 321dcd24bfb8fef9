// memset_race — does hipMemset (null stream) order with a later copy on a non-blocking
// stream? host.cpp's fixed-width context zeroed its device arena with hipMemset, then made
// its streams with hipStreamNonBlocking, and a first call's H2D copies on one of them
// filled chunk 0's column slices. If the null-stream fill can still be pending when
// hipMemset returns, and the non-blocking stream does not wait for it, the fill can land
// after the copies and zero them. That is the "first chunk of a fresh context wrong, all
// zeros" failure of rounds 5 and 6.
// Per trial:
//   1. a spin kernel on the null stream keeps it busy for ~`spin` cycles;
//   2. hipMemset(buf, 0) is timed: it returns before the spin ends (~40 ms at the default)
//      or after;
//   3. an H2D of 0xAB bytes into buf goes on a non-blocking stream, which is synchronised;
//   4. after a device sync, buf is counted for zero bytes.
// Then the fixed protocol: hipMemsetAsync on the non-blocking stream and a stream sync before
// the copy. Two more protocols keep the old hipMemset but make a call between it and the copy
// that the library's first encode makes on a fresh context (a pinned staging allocation,
// hipHostMalloc; a device allocation, hipMalloc): if such a call waits for the null stream,
// the race cannot hit through that path. The last protocol is the old library's exact
// order: hipMemset, then three non-blocking streams created, and the copy on the first. Usage: memset_race <trials> <spin cycles>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void spin_kernel(long long cycles, int* flag) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 0 && blockIdx.x == 0) *flag = 1;  // (a vector store: the kernel has finished)
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 5;
  const long long spin = argc > 2 ? atoll(argv[2]) : 100000000LL;
  const size_t n = size_t(4) << 20;
  CK(hipSetDevice(0));
  uint8_t* buf = nullptr;
  int* flag = nullptr;
  uint8_t* src = nullptr;
  CK(hipMalloc(&buf, n));
  CK(hipMalloc(&flag, sizeof(int)));
  CK(hipHostMalloc(reinterpret_cast<void**>(&src), n, hipHostMallocDefault));
  memset(src, 0xAB, n);
  std::vector<uint8_t> got(n);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const char* names[5] = {"hipMemset (null stream)", "memsetAsync on the stream + sync",
                          "hipMemset, then hipHostMalloc", "hipMemset, then hipMalloc",
                          "hipMemset, then 3 new non-blocking streams (old library order)"};
  for (int fixed = 0; fixed < 5; ++fixed) {
    for (int t = 0; t < trials; ++t) {
      CK(hipMemset(flag, 0, sizeof(int)));
      CK(hipDeviceSynchronize());
      hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, 0, spin, flag);  // the null stream
      const auto t0 = std::chrono::steady_clock::now();
      void* extra = nullptr;
      if (fixed != 1) {
        CK(hipMemset(buf, 0, n));  // the round-5/6 arena zeroing
      } else {
        CK(hipMemsetAsync(buf, 0, n, s));  // the fix: on the context's stream, waited for
        CK(hipStreamSynchronize(s));
      }
      if (fixed == 2) CK(hipHostMalloc(&extra, size_t(16) << 20, hipHostMallocPortable | hipHostMallocCoherent));
      if (fixed == 3) CK(hipMalloc(&extra, size_t(16) << 20));
      hipStream_t fresh[3] = {};
      if (fixed == 4)
        for (hipStream_t& f : fresh) CK(hipStreamCreateWithFlags(&f, hipStreamNonBlocking));
      hipStream_t cs = fixed == 4 ? fresh[0] : s;
      const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      CK(hipMemcpyAsync(buf, src, n, hipMemcpyHostToDevice, cs));  // nothing on the null stream before it
      CK(hipStreamSynchronize(cs));
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), buf, n, hipMemcpyDeviceToHost));
      if (fixed == 2) CK(hipHostFree(extra));
      if (fixed == 3) CK(hipFree(extra));
      if (fixed == 4)
        for (hipStream_t f : fresh) CK(hipStreamDestroy(f));
      size_t zeros = 0;
      for (size_t i = 0; i < n; ++i) zeros += got[i] == 0;
      printf("{\"protocol\": \"%s\", \"trial\": %d, \"memset_returned_ms\": %.3f, \"zero_bytes_after_copy\": %zu}\n",
             names[fixed], t, ms, zeros);
      fflush(stdout);
    }
  }
  return 0;
}
