// host.cpp — host-memory path of the C-ABI (include/fory_rowfmt.h, "host path").
//
// The reference path starts and ends in host memory: Encoder.encode(MemoryBuffer, T)
// appends frames to an off-heap MemoryBuffer on its way to an RPC socket and
// Encoder.decode(MemoryBuffer) reads them back (java/fory-format/.../encoder/
// Encoders.java:177-225; off-heap addresses: java/fory-core/.../memory/
// MemoryBuffer.java:287-297). A fory_host_ctx moves such host batches through
// the device kernels with a three-stream chunk pipeline: H2D of chunk k+1 ||
// kernel of chunk k || D2H of chunk k-1, double-buffered device chunks
// allocated once per context. It is a client of the device entry points in
// capi.cpp (plan_info / workspace_bytes / encode / decode / read_status).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <iterator>
#include <map>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#if defined(__x86_64__)
#include <emmintrin.h>
#endif
#include <string>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fory_rowfmt.h"

namespace fory_amd {  // scan.hip (kernels.h)
hipError_t launch_offsets_add(int32_t* offs, int64_t n, int32_t base, hipStream_t s);
hipError_t launch_bits_shift(const uint8_t* src, int64_t nbits, uint8_t* dst, int shift, hipStream_t s);
bool host_verify_from_env();  // launch_state.cpp: FORY_ROWFMT_HOST_VERIFY
}  // namespace fory_amd

namespace {


constexpr int64_t kAlign = 256;
int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

struct Slice {  // one column's device chunk buffers
  uint8_t* values = nullptr;
  uint8_t* validity = nullptr;
};

// Pinned staging of a context for caller memory that is not pinned over the whole
// copy (pageable, or a range only partly inside a registration). A ring of blocks:
// an H2D piece is memcpy'd into a block and DMA'd from it; a D2H piece is DMA'd into
// a block and memcpy'd out when the block is next needed or at the end of the call
// (drain). A block is reused only after the event of its last DMA completed, so the
// host memcpy of one piece overlaps the DMA of the others and nothing is ever copied
// by the runtime's own pageable path. Owned by one context (one call at a time): no
// lock, nothing shared across contexts or devices.
// Host memcpy of the staged copies, split over a small process-wide pool of threads: a
// pageable buffer's bytes cross host memory twice (caller <-> pinned block), and one thread
// copying them held the staged path at ~29 GB/s of PCIe (round 4).
// memcpy with non-temporal 16-byte stores: a staged piece is written once and read by
// the DMA engine (or by nobody on the host again), so the stores skip the caches'
// read-for-ownership; fenced before returning (the DMA that follows must see them).
void stream_copy(uint8_t* dst, const uint8_t* src, size_t n) {
#if defined(__x86_64__) && defined(__SSE2__)
  if (n >= 4096) {
    const size_t head = (16 - (reinterpret_cast<uintptr_t>(dst) & 15)) & 15;
    std::memcpy(dst, src, head);
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
    std::memcpy(dst + i, src + i, n - i);
    _mm_sfence();
    return;
  }
#endif
  std::memcpy(dst, src, n);
}

class CopyPool {
 public:
  static CopyPool& get() {
    static CopyPool pool;
    return pool;
  }
  void copy(void* dst, const void* src, size_t n) {
    const int parts = n >= kMinSplit && nthreads_ > 0 ? (int)std::min<size_t>(nthreads_ + 1, n / (kMinSplit / 4)) : 1;
    if (parts <= 1) {
      std::memcpy(dst, src, n);
      return;
    }
    std::unique_lock<std::mutex> lock(mu_);  // one job at a time
    if (busy_) {  // another context's job has the pool: copy on this thread rather than queue
      lock.unlock();
      stream_copy(static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n);
      return;
    }
    busy_ = true;
    dst_ = static_cast<uint8_t*>(dst);
    src_ = static_cast<const uint8_t*>(src);
    n_ = n;
    parts_ = parts;
    next_ = 1;  // part 0 is the caller's
    left_ = parts - 1;
    ++gen_;
    lock.unlock();
    work_.notify_all();
    run_part(0);
    lock.lock();
    while (next_ < parts_) {  // parts no worker picked up yet
      const int k = next_++;
      --left_;
      lock.unlock();
      run_part(k);
      lock.lock();
    }
    done_.wait(lock, [&] { return left_ == 0 && active_ == 0; });
    busy_ = false;
  }

 private:
  static constexpr size_t kMinSplit = size_t(1) << 20;
  static constexpr unsigned kMaxThreads = 15;  // a GPU's share of a host's cores (16 per MI355X)
  CopyPool() {
    const unsigned hw = std::thread::hardware_concurrency();
    nthreads_ = (int)std::min<unsigned>(kMaxThreads, hw > 1 ? hw - 1 : 0);
    for (int i = 0; i < nthreads_; ++i) threads_.emplace_back([this] { loop(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> lock(mu_);
      stop_ = true;
    }
    work_.notify_all();
    for (std::thread& t : threads_) t.join();
  }
  void run_part(int k) {
    const size_t per = ((n_ + parts_ - 1) / parts_ + 63) & ~size_t(63);  // parts x per >= n
    const size_t a = std::min(n_, per * (size_t)k), b = std::min(n_, a + per);
    if (b > a) stream_copy(dst_ + a, src_ + a, b - a);
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> lock(mu_);
    for (;;) {
      work_.wait(lock, [&] { return stop_ || (gen_ != seen && next_ < parts_); });
      if (stop_) return;
      seen = gen_;
      while (next_ < parts_) {
        const int k = next_++;
        ++active_;
        lock.unlock();
        run_part(k);
        lock.lock();
        --active_;
        --left_;
      }
      if (left_ == 0 && active_ == 0) done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable work_, done_;
  std::vector<std::thread> threads_;
  int nthreads_ = 0;
  bool busy_ = false, stop_ = false;
  uint8_t* dst_ = nullptr;
  const uint8_t* src_ = nullptr;
  size_t n_ = 0;
  int parts_ = 0, next_ = 0, left_ = 0, active_ = 0;
  uint64_t gen_ = 0;
};

#ifndef FORY_STAGE_BLOCK_MB  // (build-time A/B of the staging geometry)
#define FORY_STAGE_BLOCK_MB 16
#endif
#ifndef FORY_STAGE_BLOCKS
#define FORY_STAGE_BLOCKS 8
#endif
struct Staging {
  static constexpr size_t kBlock = size_t(FORY_STAGE_BLOCK_MB) << 20;  // a staged piece: one pool-split memcpy + one DMA
  static constexpr int kBlocks = FORY_STAGE_BLOCKS;
  uint8_t* mem = nullptr;  // kBlocks x kBlock, hipHostMalloc'd on first use
  hipEvent_t ev[kBlocks] = {};
  bool inflight[kBlocks] = {};  // ev recorded, completion not yet observed
  struct Owed { uint8_t* dst = nullptr; size_t len = 0; } owed[kBlocks];  // D2H host copies pending
  int next = 0;
  int64_t pieces = 0;  // statistics: pieces staged over the context's life
  // Small pieces (<= kSmall: the unaligned ends of registered caller buffers) are packed
  // into small buffers instead of taking a block each: per stream two buffers, filled in
  // turn; a buffer is reused only after the event of its last DMA completed. (A block per
  // 4 KiB end piece made the 104 column heads of a decode chunk wait, 8 pieces apart, for
  // the D2H stream: the host thread followed the DMA engine.)
  static constexpr size_t kSmall = size_t(64) << 10;
  static constexpr size_t kSmallBuf = size_t(2) << 20;
  static constexpr int kSmallStreams = 3;
  struct SmallOwed {
    uint8_t* dst;
    size_t at, len;
  };
  struct Small {
    hipStream_t s = nullptr;
    int cur = 0;
    size_t used[2] = {};
    hipEvent_t ev[2] = {};
    bool inflight[2] = {};
    std::vector<SmallOwed> owed[2];
  } small[kSmallStreams];
  uint8_t* smem = nullptr;  // kSmallStreams x 2 x kSmallBuf
};

}  // namespace

struct fory_host_ctx {
  const fory_plan* plan = nullptr;
  fory_plan_info info{};
  int device = 0;
  int64_t chunk = 0;
  std::vector<int32_t> width;       // per top-level column (fixed-width plans: one column per field)
  std::vector<int32_t> nullable;
  uint8_t* arena = nullptr;         // both buffers, carved
  struct Buf {
    std::vector<Slice> cols;
    uint8_t* rows = nullptr;
    void* ws = nullptr;
    int32_t* status = nullptr;
  } buf[2];
  int64_t ws_bytes = 0;
  hipStream_t s_in = nullptr, s_k = nullptr, s_out = nullptr;
  hipEvent_t ev_in[2] = {}, ev_k[2] = {}, ev_out[2] = {};
  // varlen plans: encode pipelined over two chunk slots (grown on demand), decode
  // whole batch per call (device buffers kept and grown)
  bool varlen = false;
  std::vector<int32_t> kind, parent;
  struct VarSlot {
    uint8_t* dev = nullptr;  // column slices, row offsets, workspace
    int64_t dev_bytes = 0;
    uint8_t* rows = nullptr;  // the chunk's rows / frames
    int64_t rows_bytes = 0;
    int64_t* pin = nullptr;  // pinned host copy of the chunk's row offsets
    int64_t pin_words = 0;
    bool used = false;  // events of this slot have been recorded
  } vs[2];
  hipEvent_t ev_sz[2] = {};
  int32_t* vstatus = nullptr;  // one status word per slot (sticky over a call)
  uint8_t* dbuf = nullptr;   // columns, row offsets, workspace, status
  int64_t dbuf_bytes = 0;
  uint8_t* drows = nullptr;  // rows / frames
  int64_t drows_bytes = 0;
  uint8_t* dout = nullptr;   // decode: output columns
  int64_t dout_bytes = 0;
  // decode state between host_decode_var_sizes and host_decode_var
  int64_t dec_n = -1;
  int32_t dec_frame = 0;
  std::vector<int64_t> dec_count, dec_bytes;
  std::vector<fory_column> dec_cols;
  int64_t* dec_offs = nullptr;
  void* dec_ws = nullptr;
  int32_t* dec_status = nullptr;
  Staging stage;               // pageable caller memory
  uint8_t* hpin = nullptr;     // pinned scratch: level totals, frame end, validity stash
  int64_t hpin_bytes = 0;
  // Pageable caller buffers of the current call (CallScope): each one's page-aligned
  // interior, in pieces of <= 256 MiB, is registered by the calling thread when a copy
  // first touches it and unregistered when the call returns; copies inside a registered
  // piece are direct DMAs, the buffers' unaligned heads and tails go through the staging.
  // (Round 6 first registered on a helper thread, ahead of the copies; a traced suite run
  // then faulted inside this path, and every HIP call of a context is kept on the calling
  // thread since: profiles/r06/intermittent/README.md.)
  struct Extent {
    uintptr_t base = 0, end = 0;  // the part of the caller buffer this piece covers
    uintptr_t lo = 0, hi = 0;     // its page-aligned interior
    int state = 0;                // 0 not registered yet, 1 registered by this call, 2 declined
  };
  std::vector<Extent> ext;
  int64_t reg_calls = 0, reg_bytes = 0;  // statistics: call-scoped registrations over the context's life
  double reg_ms = 0;
  // FORY_ROWFMT_HOST_VERIFY=1 (read at context creation; tests / diagnosis only): after
  // each chunk's host-to-device copies the device bytes are read back and compared with
  // the caller's; a mismatch fails the call naming the piece and the source it matches.
  bool verify = false;
  struct VPiece {
    const uint8_t* dev;
    const uint8_t* host;
    size_t bytes;
    const char* what;
    int64_t seq;
  };
  std::vector<VPiece> vcur, vprev;
  int64_t vseq = 0;
  uint8_t* vpin = nullptr;  // pinned read-back buffer of the verify mode
  size_t vpin_bytes = 0;
};

namespace {

int fail_host(int code, const std::string& msg);

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return FORY_OK;
  return fail_host(FORY_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

}  // namespace

// Library-internal helpers of capi.cpp (not in the public header): last_error
// is thread-local there; column widths/nullability of a fixed-width plan.
extern "C" int fory_rowfmt_internal_set_error(int code, const char* msg);
extern "C" void fory_rowfmt_internal_retire_stream(void* stream);
extern "C" int fory_rowfmt_internal_column_layout(const fory_plan* plan, int32_t* width, int32_t* nullable);
extern "C" int fory_rowfmt_internal_node_layout(const fory_plan* plan, int32_t* kind, int32_t* width,
                                                int32_t* nullable, int32_t* parent);

namespace {

int fail_host(int code, const std::string& msg) { return fory_rowfmt_internal_set_error(code, msg.c_str()); }

// Ranges registered through fory_rowfmt_host_register: base -> (bytes, the device
// address of base). Copies inside one of them find their mapping here, without the
// four runtime pointer queries of mapped_range (each tens of microseconds: a chunk's
// 104 column copies were issued ~110 us apart, the DMA idle in between).
struct Reg {
  size_t bytes;
  uint8_t* dev;
};
std::mutex g_reg_mu;
std::map<uintptr_t, Reg> g_regs;
// Call-scoped registrations (fory_host_ctx::ext): interior start -> (bytes, device
// address of the start, null while the registration is in progress; owning context).
// Only the owner's copies use them: another context's copy over one is staged, since the
// owner unregisters it when its call returns, whatever that other copy's DMA is doing.
struct TmpReg {
  size_t bytes;
  uint8_t* dev;
  const fory_host_ctx* owner;
};
std::map<uintptr_t, TmpReg> g_tmp;

std::string hex(uintptr_t a) {
  char b[32];
  std::snprintf(b, sizeof b, "0x%llx", (unsigned long long)a);
  return b;
}

// Does the runtime still treat host address p as registered (pinned, device-mapped)?
bool still_mapped(const void* p) {
  hipPointerAttribute_t a{};
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type != hipMemoryTypeUnregistered && a.devicePointer != nullptr;
}

int64_t validity_bytes(int64_t rows) { return ((rows + 7) / 8 + 3) / 4 * 4; }

// Is [p, p + bytes) pinned as ONE mapping, so that an async DMA may read or write it
// directly? Round 2 judged a copy by its first byte only: a range that begins inside
// a registration (hipHostRegister / fory_rowfmt_host_register, or hipHostMalloc) and
// runs past its end was handed to hipMemcpyAsync as if pinned, and the DMA then
// reaches host pages the device has no mapping for. Now the first and the last byte
// must both be pinned, map to device addresses exactly bytes - 1 apart, and lie in
// the allocation range the runtime reports. Anything else is staged (Staging).
uint8_t* mapped_range(const void* p, size_t bytes, const fory_host_ctx* owner = nullptr);
bool pinned_range(const void* p, size_t bytes, const fory_host_ctx* owner = nullptr) {
  return mapped_range(p, bytes, owner) != nullptr;
}

// The device address of host byte p when [p, p + bytes) is pinned as one mapping (the
// conditions above), else nullptr.
uint8_t* mapped_range(const void* p, size_t bytes, const fory_host_ctx* owner) {
  if (!p || bytes == 0) return nullptr;
  {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    std::lock_guard<std::mutex> lock(g_reg_mu);
#ifndef FORY_AB_MAPPING_QUERIES  // (build-time A/B: -D it to resolve every copy by runtime queries, as round 4)
    // inside a range this library registered: its mapping is known
    auto it = g_regs.upper_bound(a);
    if (it != g_regs.begin()) {
      --it;
      if (a >= it->first && a + bytes <= it->first + it->second.bytes) return it->second.dev + (a - it->first);
    }
#endif
    // a call-scoped registration: its owner's copies inside it are direct; any other
    // copy touching one is staged (entries are disjoint and sorted: walk back from the
    // last one starting inside the range until one ends before it)
    auto jt = g_tmp.upper_bound(a + bytes - 1);
    if (jt != g_tmp.begin()) {
      --jt;
      if (jt->first + jt->second.bytes > a) {
        if (owner && jt->second.owner == owner && jt->second.dev && a >= jt->first &&
            a + bytes <= jt->first + jt->second.bytes)
          return jt->second.dev + (a - jt->first);
        return nullptr;
      }
    }
  }
  const uint8_t* first = static_cast<const uint8_t*>(p);
  const uint8_t* last = first + (bytes - 1);
  hipPointerAttribute_t a{}, b{};
  if (hipPointerGetAttributes(&a, first) != hipSuccess || hipPointerGetAttributes(&b, last) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a.type == hipMemoryTypeUnregistered || b.type == hipMemoryTypeUnregistered) return nullptr;
  if (!a.devicePointer || !b.devicePointer ||
      static_cast<const uint8_t*>(b.devicePointer) - static_cast<const uint8_t*>(a.devicePointer) !=
          static_cast<std::ptrdiff_t>(bytes - 1))
    return nullptr;
  void* start = nullptr;
  size_t size = 0;
  if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, const_cast<uint8_t*>(first)) ==
          hipSuccess &&
      hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, const_cast<uint8_t*>(first)) == hipSuccess &&
      start && size) {
    // the runtime may report the range in host or in device addresses: either must hold the copy
    const uint8_t* s0 = static_cast<const uint8_t*>(start);
    const uint8_t* d0 = static_cast<const uint8_t*>(a.devicePointer);
    const bool host_in = first >= s0 && last < s0 + size;
    const bool dev_in = d0 >= s0 && d0 + (bytes - 1) < s0 + size;
    if (!host_in && !dev_in) return nullptr;
  } else {
    (void)hipGetLastError();
  }
  return static_cast<uint8_t*>(a.devicePointer);
}

int stage_alloc(Staging& st) {
  if (st.mem) return FORY_OK;
  // coherent (fine-grained) host memory: the blocks are rewritten by the host between
  // DMAs and re-allocated across contexts, so no device-side cached line of an earlier
  // use may serve a later copy
  int rc = hip_check(hipHostMalloc(reinterpret_cast<void**>(&st.mem), Staging::kBlock * Staging::kBlocks,
                                   hipHostMallocPortable | hipHostMallocCoherent),
                     "hipHostMalloc(staging)");
  for (int j = 0; j < Staging::kBlocks && !rc; ++j)
    if (!st.ev[j]) rc = hip_check(hipEventCreateWithFlags(&st.ev[j], hipEventDisableTiming), "hipEventCreate");
  return rc;
}

// After a failed wait on a staging event: no owed D2H copy of this call may be made
// later (its caller buffers may be gone by the context's next call), and no block is
// waited for again. The context's next call starts with clean staging.
void stage_abandon(Staging& st) {
  for (int j = 0; j < Staging::kBlocks; ++j) {
    st.inflight[j] = false;
    st.owed[j] = Staging::Owed{};
  }
  for (auto& sm : st.small)
    for (int b = 0; b < 2; ++b) sm.inflight[b] = false, sm.owed[b].clear(), sm.used[b] = 0;
}

uint8_t* small_buf(Staging& st, int k, int b) { return st.smem + ((size_t)k * 2 + b) * Staging::kSmallBuf; }

// Small buffer b of stream slot k free again: its last DMA done, its owed D2H copies made.
int small_retire(Staging& st, int k, int b) {
  Staging::Small& sm = st.small[k];
  if (sm.inflight[b]) {
    int rc = hip_check(hipEventSynchronize(sm.ev[b]), "hipEventSynchronize(small staging)");
    if (rc) {
      stage_abandon(st);
      return rc;
    }
    sm.inflight[b] = false;
  }
  for (const auto& o : sm.owed[b]) std::memcpy(o.dst, small_buf(st, k, b) + o.at, o.len);
  sm.owed[b].clear();
  sm.used[b] = 0;
  return FORY_OK;
}

// A small piece on stream s through the stream's small buffers.
int stage_small(Staging& st, void* dst, const void* src, size_t len, hipMemcpyKind kind, hipStream_t s,
                const char* what) {
  int rc = FORY_OK;
  if (!st.smem) {
    rc = hip_check(hipHostMalloc(reinterpret_cast<void**>(&st.smem), Staging::kSmallBuf * 2 * Staging::kSmallStreams,
                                 hipHostMallocPortable | hipHostMallocCoherent),
                   "hipHostMalloc(small staging)");
    if (rc) return rc;
  }
  int k = 0;
  while (k < Staging::kSmallStreams && st.small[k].s && st.small[k].s != s) ++k;
  if (k == Staging::kSmallStreams) {  // (more streams than slots: slot 0 is drained and taken over)
    k = 0;
    for (int b = 0; b < 2 && !rc; ++b) rc = small_retire(st, 0, b);
    if (rc) return rc;
    st.small[0].s = nullptr;
  }
  Staging::Small& sm = st.small[k];
  if (!sm.s) {
    sm.s = s;
    for (int b = 0; b < 2 && !rc; ++b)
      if (!sm.ev[b]) rc = hip_check(hipEventCreateWithFlags(&sm.ev[b], hipEventDisableTiming), "hipEventCreate");
    if (rc) return rc;
  }
  const size_t need = (len + 15) & ~size_t(15);
  if (sm.used[sm.cur] + need > Staging::kSmallBuf) {  // the other buffer, once its last DMA is done
    sm.cur ^= 1;
    rc = small_retire(st, k, sm.cur);
    if (rc) return rc;
  }
  const int b = sm.cur;
  const size_t at = sm.used[b];
  uint8_t* p = small_buf(st, k, b) + at;
  if (kind == hipMemcpyHostToDevice) {
    std::memcpy(p, src, len);
    rc = hip_check(hipMemcpyAsync(dst, p, len, kind, s), what);
  } else {
    rc = hip_check(hipMemcpyAsync(p, src, len, kind, s), what);
    if (!rc) sm.owed[b].push_back(Staging::SmallOwed{static_cast<uint8_t*>(dst), at, len});
  }
  if (!rc) rc = hip_check(hipEventRecord(sm.ev[b], s), "hipEventRecord(small staging)");
  if (!rc) sm.inflight[b] = true;
  sm.used[b] += need;
  ++st.pieces;
  return rc;
}

// Block j free for a new piece: its last DMA done, an owed D2H host copy made.
int stage_retire(Staging& st, int j) {
  if (st.inflight[j]) {
    int rc = hip_check(hipEventSynchronize(st.ev[j]), "hipEventSynchronize(staging)");
    if (rc) {
      stage_abandon(st);
      return rc;
    }
    st.inflight[j] = false;
  }
  if (st.owed[j].dst) {
    CopyPool::get().copy(st.owed[j].dst, st.mem + (size_t)j * Staging::kBlock, st.owed[j].len);
    st.owed[j] = Staging::Owed{};
  }
  return FORY_OK;
}

// Every staged piece complete, every owed D2H copy in caller memory (oldest first).
int stage_drain(Staging& st) {
  if (st.smem)
    for (int k = 0; k < Staging::kSmallStreams; ++k) {
      for (int i = 0; i < 2; ++i) {
        const int rc = small_retire(st, k, st.small[k].cur ^ 1 ^ i);  // the older buffer first
        if (rc) return rc;
      }
      st.small[k].s = nullptr;  // (streams are the context's; a slot is re-bound per call)
      st.small[k].cur = 0;
    }
  if (!st.mem) return FORY_OK;
  for (int i = 0; i < Staging::kBlocks; ++i) {
    const int rc = stage_retire(st, (st.next + i) % Staging::kBlocks);
    if (rc) return rc;  // (stage_abandon cleared every block)
  }
  return FORY_OK;
}

// A copy through the context's staging: H2D pieces are in pinned memory before this
// returns (the caller may reuse its buffer); D2H pieces land in caller memory at the next
// stage_drain (sync_all).
int hcopy_staged(fory_host_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s,
                 const char* what);

// Call-scoped registration of caller buffer e's page-aligned interior (first copy that
// touches it). Declined -- the buffer's pieces stay staged -- when the interior overlaps
// a registration of this library (fory_rowfmt_host_register or another call's), when the
// runtime already maps either end (the caller registered it: mapped_range takes such
// copies whole) or when hipHostRegister refuses it. Registering costs ~4-11 ms per GiB of
// touched pages on MI355X hosts against ~18 ms per GiB of DMA at 57 GB/s
// (scripts/microbench/reg_probe.hip, profiles/r06/host/), and no byte crosses host memory
// a second time.
// Returns the piece's new state (1 registered, 2 declined).
int ext_register_state(fory_host_ctx* c, fory_host_ctx::Extent& e) {
  const size_t len = e.hi - e.lo;
  {
    std::lock_guard<std::mutex> lock(g_reg_mu);
    for (const auto& r : g_regs)
      if (e.lo < r.first + r.second.bytes && r.first < e.hi) return 2;
    auto jt = g_tmp.upper_bound(e.hi - 1);
    if (jt != g_tmp.begin() && std::prev(jt)->first + std::prev(jt)->second.bytes > e.lo) return 2;
    g_tmp[e.lo] = TmpReg{len, nullptr, c};  // reserved: nobody's copies use it yet
  }
  auto drop = [&]() {
    std::lock_guard<std::mutex> lock(g_reg_mu);
    g_tmp.erase(e.lo);
    return 2;
  };
  void* lo = reinterpret_cast<void*>(e.lo);
  void* last = reinterpret_cast<void*>(e.hi - 1);
  if (still_mapped(lo) || still_mapped(last)) return drop();
  const auto t0 = std::chrono::steady_clock::now();
  if (hipHostRegister(lo, len, hipHostRegisterDefault) != hipSuccess) {
    (void)hipGetLastError();
    return drop();
  }
  hipPointerAttribute_t a{}, z{};
  if (hipPointerGetAttributes(&a, lo) != hipSuccess || hipPointerGetAttributes(&z, last) != hipSuccess ||
      !a.devicePointer || !z.devicePointer ||
      static_cast<uint8_t*>(z.devicePointer) - static_cast<uint8_t*>(a.devicePointer) != (std::ptrdiff_t)(len - 1)) {
    (void)hipGetLastError();
    (void)hipHostUnregister(lo);
    return drop();
  }
  c->reg_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  ++c->reg_calls;
  c->reg_bytes += (int64_t)len;
  std::lock_guard<std::mutex> lock(g_reg_mu);
  g_tmp[e.lo].dev = static_cast<uint8_t*>(a.devicePointer);
  return 1;
}

// The registration state of piece e, registering it on first touch.
int ext_state(fory_host_ctx* c, fory_host_ctx::Extent& e) {
  if (!e.state) e.state = ext_register_state(c, e);
  return e.state;
}

// One copy between caller host memory and the device, queued on stream s. Pinned over
// its whole range (or inside this call's registration of the caller buffer holding it):
// one async DMA. Inside a pageable caller buffer declared for the call (CallScope): the
// buffer's interior registered on first touch, the copy split into a direct middle and
// staged unaligned ends. Anything else goes through the context's staging.
int hcopy(fory_host_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s,
          const char* what) {
  if (bytes == 0) return FORY_OK;
  const bool h2d = kind == hipMemcpyHostToDevice;
  const uint8_t* hp = static_cast<const uint8_t*>(h2d ? src : dst);
  if (c->verify && h2d) c->vcur.push_back({static_cast<const uint8_t*>(dst), hp, bytes, what, c->vseq++});
  if (pinned_range(hp, bytes, c)) return hip_check(hipMemcpyAsync(dst, src, bytes, kind, s), what);
  const uintptr_t a = reinterpret_cast<uintptr_t>(hp), z = a + bytes;
  uint8_t* d8 = static_cast<uint8_t*>(h2d ? dst : const_cast<void*>(src));  // the device side
  auto piece = [&](uintptr_t u0, uintptr_t u1, bool direct) -> int {
    if (u1 <= u0) return FORY_OK;
    uint8_t* hptr = reinterpret_cast<uint8_t*>(u0);
    uint8_t* dptr = d8 + (u0 - a);
    void* pd = h2d ? static_cast<void*>(dptr) : static_cast<void*>(hptr);
    const void* ps = h2d ? static_cast<const void*>(hptr) : static_cast<const void*>(dptr);
    if (direct) return hip_check(hipMemcpyAsync(pd, ps, u1 - u0, kind, s), what);
    return hcopy_staged(c, pd, ps, u1 - u0, kind, s, what);
  };
  // the registered pieces of declared caller buffers over [a, z), in address order (a
  // buffer's pieces were declared in order and abut): one direct DMA per piece (a DMA
  // may not run past a registration), the gaps -- unaligned ends, declined pieces -- staged
  uintptr_t cur = a;
  int rc = FORY_OK;
  for (fory_host_ctx::Extent& e : c->ext) {
    if (rc || cur >= z) break;
    if (e.base >= z || e.end <= cur || e.lo >= z || e.hi <= cur) continue;
    if (ext_state(c, e) != 1) continue;
    const uintptr_t x0 = std::max(cur, e.lo), x1 = std::min(z, e.hi);
    if (x1 <= x0) continue;
    rc = piece(cur, x0, false);
    if (!rc) rc = piece(x0, x1, true);
    cur = x1;
  }
  if (!rc) rc = piece(cur, z, false);
  return rc;
}

int hcopy_staged(fory_host_ctx* c, void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s,
                 const char* what) {
  const bool h2d = kind == hipMemcpyHostToDevice;
  Staging& st = c->stage;
  if (bytes <= Staging::kSmall) return stage_small(st, dst, src, bytes, kind, s, what);
  int rc = stage_alloc(st);
  for (size_t off = 0; off < bytes && !rc; off += Staging::kBlock) {
    const size_t len = std::min(bytes - off, Staging::kBlock);
    const int j = st.next;
    st.next = (st.next + 1) % Staging::kBlocks;
    rc = stage_retire(st, j);
    if (rc) break;
    uint8_t* blk = st.mem + (size_t)j * Staging::kBlock;
    if (h2d) {
      CopyPool::get().copy(blk, static_cast<const uint8_t*>(src) + off, len);
      rc = hip_check(hipMemcpyAsync(static_cast<uint8_t*>(dst) + off, blk, len, kind, s), what);
    } else {
      rc = hip_check(hipMemcpyAsync(blk, static_cast<const uint8_t*>(src) + off, len, kind, s), what);
      if (!rc) st.owed[j] = Staging::Owed{static_cast<uint8_t*>(dst) + off, len};
    }
    if (!rc) rc = hip_check(hipEventRecord(st.ev[j], s), "hipEventRecord(staging)");
    if (!rc) st.inflight[j] = true;
    ++st.pieces;
  }
  return rc;
}

// Context-owned pinned scratch of at least `bytes` (grown, never per call).
int ensure_hpin(fory_host_ctx* c, int64_t bytes) {
  if (bytes <= c->hpin_bytes) return FORY_OK;
  if (c->hpin) (void)hipHostFree(c->hpin);
  c->hpin = nullptr;
  c->hpin_bytes = 0;
  const int64_t sz = align_up(bytes + bytes / 2);
  int rc = hip_check(hipHostMalloc(reinterpret_cast<void**>(&c->hpin), (size_t)sz, hipHostMallocCoherent),
                     "hipHostMalloc(ctx scratch)");
  if (!rc) c->hpin_bytes = sz;
  return rc;
}

// The caller buffers of one call: declared at the call's start (call_extent), each
// registered on first touch (hcopy -> ext_register); when the call returns, every stream
// is drained (normally done already by sync_all) and every registration of the call
// removed, so no caller page stays pinned past the call and no later copy can take a
// mapping of it for a direct DMA.
#ifndef FORY_REG_MIN_KB  // (the CPU mock test, tests/c/host_copy_mock.cpp, shrinks both)
#define FORY_REG_MIN_KB 4096
#endif
#ifndef FORY_REG_PIECE_KB
#define FORY_REG_PIECE_KB (256 * 1024)
#endif
constexpr size_t kRegMin = size_t(FORY_REG_MIN_KB) << 10;  // smaller interiors stay staged

constexpr uintptr_t kRegPiece = uintptr_t(FORY_REG_PIECE_KB) << 10;  // registration granularity of big buffers

void call_extent(fory_host_ctx* c, const void* p, int64_t bytes) {
  if (!p || bytes <= 0) return;
  const uintptr_t base = reinterpret_cast<uintptr_t>(p), end = base + (uintptr_t)bytes;
  const uintptr_t lo = (base + 4095) & ~uintptr_t(4095), hi = end & ~uintptr_t(4095);
  if (hi <= lo || hi - lo < kRegMin) return;
  for (const auto& o : c->ext)
    if (lo < o.hi && o.lo < hi) return;  // (overlapping caller buffers: the first one declared)
  for (uintptr_t x = lo; x < hi; x += kRegPiece) {
    fory_host_ctx::Extent& e = c->ext.emplace_back();
    e.lo = x;
    e.hi = std::min(hi, x + kRegPiece);
    e.base = x == lo ? base : x;
    e.end = e.hi == hi ? end : e.hi;
  }
}

struct CallScope {
  fory_host_ctx* c;
  explicit CallScope(fory_host_ctx* ctx) : c(ctx) {
    c->ext.clear();
    c->vcur.clear();
    c->vprev.clear();
  }
  ~CallScope() {
    // whatever path the call returns by (an error return skips sync_all): every queued copy
    // done and every owed D2H host copy made while the caller's buffers are still this
    // call's, then the call's registrations removed. After a normal return both are no-ops.
    for (hipStream_t s : {c->s_in, c->s_k, c->s_out})
      if (s) (void)hipStreamSynchronize(s);
    if (stage_drain(c->stage)) stage_abandon(c->stage);
    for (const auto& e : c->ext) {
      if (e.state != 1) continue;
      (void)hipHostUnregister(reinterpret_cast<void*>(e.lo));
      (void)hipGetLastError();
      std::lock_guard<std::mutex> lock(g_reg_mu);
      g_tmp.erase(e.lo);
    }
    c->ext.clear();
  }
};

// FORY_ROWFMT_HOST_VERIFY: the device bytes of every host-to-device piece queued since the
// last check, read back and compared with the caller's bytes once `s` (the stream they
// were queued on) has drained. A wrong piece fails the call, naming it, the first wrong
// byte and -- when the device bytes equal the source of another piece of this chunk or
// the chunk before -- that piece (a staging block or device buffer handed on too early).
int verify_pieces(fory_host_ctx* c, hipStream_t s, int64_t chunk) {
  if (!c->verify) return FORY_OK;
  int rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize(verify)");
  for (size_t i = 0; i < c->vcur.size() && !rc; ++i) {
    const auto& v = c->vcur[i];
    if (v.bytes > c->vpin_bytes) {  // read back through pinned memory (no pageable runtime copy)
      if (c->vpin) (void)hipHostFree(c->vpin);
      c->vpin = nullptr, c->vpin_bytes = 0;
      rc = hip_check(hipHostMalloc(reinterpret_cast<void**>(&c->vpin), v.bytes, hipHostMallocCoherent),
                     "hipHostMalloc(verify)");
      if (rc) break;
      c->vpin_bytes = v.bytes;
    }
    uint8_t* got = c->vpin;
    rc = hip_check(hipMemcpyAsync(got, v.dev, v.bytes, hipMemcpyDeviceToHost, s), "hipMemcpyAsync(verify)");
    if (!rc) rc = hip_check(hipStreamSynchronize(s), "hipStreamSynchronize(verify)");
    if (rc || !std::memcmp(got, v.host, v.bytes)) continue;
    size_t first = 0, wrong = 0;
    while (got[first] == v.host[first]) ++first;
    for (size_t b = 0; b < v.bytes; ++b) wrong += got[b] != v.host[b];
    std::string like = "no other piece's source";
    for (const auto* list : {&c->vcur, &c->vprev})
      for (const auto& o : *list)
        if (o.seq != v.seq && o.bytes >= 64 && !std::memcmp(got + first, o.host + std::min(first, o.bytes - 64), 64))
          like = "piece " + std::to_string(o.seq) + " (" + o.what + ", " + std::to_string(o.bytes) + " bytes)";
    rc = fail_host(FORY_ERR_DEVICE, "host verify: chunk " + std::to_string(chunk) + " piece " + std::to_string(v.seq) +
                                        " (" + v.what + ", " + std::to_string(v.bytes) + " bytes): " +
                                        std::to_string(wrong) + " device bytes differ from the caller's, the first at " +
                                        std::to_string(first) + "; the device bytes there match " + like);
  }
  c->vprev.swap(c->vcur);
  c->vcur.clear();
  return rc;
}

// End of a pipelined call: every stream of the context drained, the first error
// reported (an asynchronous kernel fault surfaces in the call that caused it, not in
// the context's next call), and every staged D2H piece in caller memory.
int sync_all(fory_host_ctx* c) {
  int rc = hip_check(hipStreamSynchronize(c->s_out), "hipStreamSynchronize(out)");
  const int rk = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize(kernels)");
  const int ri = hip_check(hipStreamSynchronize(c->s_in), "hipStreamSynchronize(in)");
  if (rc || rk || ri) {  // (the first failure keeps the error message; nothing staged is owed any more)
    stage_abandon(c->stage);
    const int first = rc ? rc : (rk ? rk : ri);
    return first;
  }
  return stage_drain(c->stage);
}

// Chunk k's row range.
void chunk_range(const fory_host_ctx* c, int64_t n, int64_t k, int64_t* a, int64_t* rows) {
  *a = k * c->chunk;
  *rows = n - *a < c->chunk ? n - *a : c->chunk;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_ctx_create(const fory_plan* plan, int32_t device, int64_t chunk_rows,
                                fory_host_ctx** out) {
  if (!out) return fail_host(FORY_ERR_INVALID_ARGUMENT, "out is null");
  *out = nullptr;
  if (!plan) return fail_host(FORY_ERR_INVALID_ARGUMENT, "plan is null");
  fory_plan_info info{};
  int rc = fory_rowfmt_plan_info(plan, &info);
  if (rc) return rc;
  if (chunk_rows <= 0) chunk_rows = 1 << 20;
  chunk_rows = (chunk_rows + 63) / 64 * 64;  // whole 64-record tiles: validity slices are byte aligned
  if (!info.fixed_width) {  // varlen: fory_rowfmt_host_encode_var / host_decode_var_sizes / host_decode_var
    fory_host_ctx* c = new fory_host_ctx();
    c->plan = plan;
    c->info = info;
    c->device = device;
    c->chunk = chunk_rows;
    c->varlen = true;
    c->verify = fory_amd::host_verify_from_env();
    c->kind.resize(info.num_columns);
    c->parent.resize(info.num_columns);
    c->width.resize(info.num_columns);
    c->nullable.resize(info.num_columns);
    fory_rowfmt_internal_node_layout(plan, c->kind.data(), c->width.data(), c->nullable.data(), c->parent.data());
    rc = hip_check(hipSetDevice(device), "hipSetDevice");
    for (hipStream_t* s : {&c->s_in, &c->s_k, &c->s_out})
      if (!rc) rc = hip_check(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate");
    for (int b = 0; b < 2 && !rc; ++b)
      for (hipEvent_t* e : {&c->ev_in[b], &c->ev_k[b], &c->ev_out[b], &c->ev_sz[b]})
        if (!rc) rc = hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
    if (!rc) rc = hip_check(hipMalloc(&c->vstatus, kAlign), "hipMalloc(status)");
    if (rc) {
      fory_rowfmt_host_ctx_destroy(c);
      return rc;
    }
    *out = c;
    return FORY_OK;
  }
  fory_host_ctx* c = new fory_host_ctx();
  c->plan = plan;
  c->info = info;
  c->device = device;
  c->chunk = chunk_rows;
  c->verify = fory_amd::host_verify_from_env();
  rc = hip_check(hipSetDevice(device), "hipSetDevice");
  if (rc) {
    delete c;
    return rc;
  }
  c->width.resize(info.num_columns);
  c->nullable.resize(info.num_columns);
  fory_rowfmt_internal_column_layout(plan, c->width.data(), c->nullable.data());  // pre-order = schema order
  const int64_t stride = info.fixed_size + 12;  // room for frames too
  c->ws_bytes = fory_rowfmt_workspace_bytes(plan, chunk_rows);
  int64_t per = 0;
  for (int i = 0; i < info.num_columns; ++i)
    per += align_up(c->width[i] * chunk_rows) + (c->nullable[i] ? align_up(validity_bytes(chunk_rows)) : 0);
  per += align_up(stride * chunk_rows) + align_up(c->ws_bytes) + kAlign;
  rc = hip_check(hipMalloc(&c->arena, (size_t)(2 * per)), "hipMalloc(host ctx chunk buffers)");
  if (rc) {
    delete c;
    return rc;
  }
  for (int b = 0; b < 2; ++b) {
    uint8_t* p = c->arena + b * per;
    c->buf[b].cols.resize(info.num_columns);
    for (int i = 0; i < info.num_columns; ++i) {
      c->buf[b].cols[i].values = p;
      p += align_up(c->width[i] * chunk_rows);
      if (c->nullable[i]) {
        c->buf[b].cols[i].validity = p;
        p += align_up(validity_bytes(chunk_rows));
      }
    }
    c->buf[b].rows = p;
    p += align_up(stride * chunk_rows);
    c->buf[b].ws = p;
    p += align_up(c->ws_bytes);
    c->buf[b].status = reinterpret_cast<int32_t*>(p);
  }
  for (hipStream_t* s : {&c->s_in, &c->s_k, &c->s_out})
    if (!rc) rc = hip_check(hipStreamCreateWithFlags(s, hipStreamNonBlocking), "hipStreamCreate");
  // The arena is zeroed on the context's own stream and waited for here. Until round 6 this
  // was a hipMemset on the null stream, which non-blocking streams do not wait for, and it
  // may still run when hipMemset returns. A first call's H2D copies on s_in could then land
  // before the fill and be zeroed by it: chunk 0's kernels read zero columns. That is the
  // "first chunk of a fresh context wrong" failure of rounds 5 and 6
  // (profiles/r06/intermittent/README.md §6).
  if (!rc) rc = hip_check(hipMemsetAsync(c->arena, 0, (size_t)(2 * per), c->s_in), "hipMemsetAsync(arena)");
  if (!rc) rc = hip_check(hipStreamSynchronize(c->s_in), "hipStreamSynchronize(arena)");
  for (int b = 0; b < 2 && !rc; ++b)
    for (hipEvent_t* e : {&c->ev_in[b], &c->ev_k[b], &c->ev_out[b]})
      if (!rc) rc = hip_check(hipEventCreateWithFlags(e, hipEventDisableTiming), "hipEventCreate");
  if (rc) {
    fory_rowfmt_host_ctx_destroy(c);
    return rc;
  }
  *out = c;
  return FORY_OK;
}

void fory_rowfmt_host_ctx_destroy(fory_host_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->s_in) (void)hipStreamSynchronize(c->s_in);
  if (c->s_k) (void)hipStreamSynchronize(c->s_k);
  if (c->s_out) (void)hipStreamSynchronize(c->s_out);
  for (int b = 0; b < 2; ++b) {
    for (hipEvent_t e : {c->ev_in[b], c->ev_k[b], c->ev_out[b], c->ev_sz[b]})
      if (e) (void)hipEventDestroy(e);
    for (uint8_t* p : {c->vs[b].dev, c->vs[b].rows})
      if (p) (void)hipFree(p);
    if (c->vs[b].pin) (void)hipHostFree(c->vs[b].pin);
  }
  for (hipStream_t s : {c->s_in, c->s_k, c->s_out})
    if (s) {
      fory_rowfmt_internal_retire_stream(s);
      (void)hipStreamDestroy(s);
    }
  if (c->arena) (void)hipFree(c->arena);
  if (c->vstatus) (void)hipFree(c->vstatus);
  for (uint8_t* b : {c->dbuf, c->drows, c->dout})
    if (b) (void)hipFree(b);
  for (hipEvent_t e : c->stage.ev)
    if (e) (void)hipEventDestroy(e);
  if (c->stage.mem) (void)hipHostFree(c->stage.mem);
  for (auto& sm : c->stage.small)
    for (hipEvent_t e : sm.ev)
      if (e) (void)hipEventDestroy(e);
  if (c->stage.smem) (void)hipHostFree(c->stage.smem);
  if (c->hpin) (void)hipHostFree(c->hpin);
  if (c->vpin) (void)hipHostFree(c->vpin);
  delete c;
}

int fory_rowfmt_host_register(void* host_ptr, int64_t bytes) {
  if (!host_ptr || bytes <= 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "null pointer or empty range");
  const uintptr_t b = reinterpret_cast<uintptr_t>(host_ptr), e = b + (uintptr_t)bytes;
  std::lock_guard<std::mutex> lock(g_reg_mu);
  // the same bytes twice: refused (one of the two unregisters would leave the runtime
  // mapping bytes the other still counts on; copies are judged by whole ranges,
  // pinned_range). Ranges that only share a page are fine: each registration pins the page.
  for (const auto& r : g_regs)
    if (b < r.first + r.second.bytes && r.first < e)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "range overlaps a registered range at " + hex(r.first) + " (" +
                                                      std::to_string(r.second.bytes) + " bytes)");
  int rc = hip_check(hipHostRegister(host_ptr, (size_t)bytes, hipHostRegisterDefault), "hipHostRegister");
  if (rc) return rc;
  // its device mapping, checked at both ends like mapped_range does for other memory
  hipPointerAttribute_t a{}, z{};
  const uint8_t* last = static_cast<const uint8_t*>(host_ptr) + (bytes - 1);
  if (hipPointerGetAttributes(&a, host_ptr) != hipSuccess || hipPointerGetAttributes(&z, last) != hipSuccess ||
      !a.devicePointer || !z.devicePointer ||
      static_cast<const uint8_t*>(z.devicePointer) - static_cast<const uint8_t*>(a.devicePointer) != bytes - 1) {
    (void)hipGetLastError();
    (void)hipHostUnregister(host_ptr);
    return fail_host(FORY_ERR_DEVICE, "registered range has no contiguous device mapping");
  }
  g_regs[b] = Reg{(size_t)bytes, static_cast<uint8_t*>(a.devicePointer)};
  return FORY_OK;
}

int fory_rowfmt_host_unregister(void* host_ptr) {
  if (!host_ptr) return fail_host(FORY_ERR_INVALID_ARGUMENT, "null pointer");
  const uintptr_t b = reinterpret_cast<uintptr_t>(host_ptr);
  std::lock_guard<std::mutex> lock(g_reg_mu);
  auto it = g_regs.find(b);
  if (it == g_regs.end())
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "not the start of a range fory_rowfmt_host_register registered");
  const size_t bytes = it->second.bytes;
  int rc = hip_check(hipHostUnregister(host_ptr), "hipHostUnregister");
  if (rc) return rc;  // (still registered: kept in the table)
  g_regs.erase(it);
  // the runtime must no longer map either end of the range: a copy through it would be
  // handed to the DMA engine as pinned memory the device no longer maps
  if (still_mapped(host_ptr) || still_mapped(static_cast<uint8_t*>(host_ptr) + (bytes - 1)))
    return fail_host(FORY_ERR_DEVICE, "range still reads as registered after hipHostUnregister");
  return FORY_OK;
}

int fory_rowfmt_internal_host_registered_ranges(void) {
  std::lock_guard<std::mutex> lock(g_reg_mu);
  return (int)g_regs.size();
}

}  // extern "C"

namespace {

// Host output windows: window w receives rows [first[w], first[w+1]) of the batch
// (whole rows/frames only), at most cap[w] bytes. One window of the caller's
// capacity is the contiguous MemoryBuffer of host_encode / host_encode_var.
struct OutWindows {
  std::vector<uint8_t*> ptr;
  std::vector<int64_t> cap;
  std::vector<int64_t> first;  // size() + 1 entries once split
};

// Greedy split (a MemoryBuffer is int-sized, MemoryBuffer.java:87: the JNI side
// fills one buffer with whole frames, then the next): window w takes rows while
// they fit its capacity. Offsets from `offs` (n+1, host) or i * stride. A window too
// small for the next row stays empty; running out of windows is FORY_ERR_CAPACITY.
int split_rows(const int64_t* offs, int64_t stride, int64_t n, OutWindows* W) {
  const int64_t nw = (int64_t)W->cap.size();
  W->first.assign((size_t)nw + 1, n);
  auto at = [&](int64_t i) { return offs ? offs[i] : i * stride; };
  int64_t start = 0;
  for (int64_t w = 0; w < nw; ++w) {
    W->first[(size_t)w] = start;
    if (start >= n) continue;
    const int64_t limit = at(start) + W->cap[(size_t)w];
    int64_t lo = start, hi = n;  // largest e in [start, n] with at(e) <= limit
    while (lo < hi) {
      const int64_t mid = hi - (hi - lo) / 2;
      if (at(mid) <= limit) lo = mid;
      else hi = mid - 1;
    }
    start = lo;
  }
  W->first[(size_t)nw] = start;
  if (start < n)
    return fail_host(FORY_ERR_CAPACITY, "output windows hold " + std::to_string(start) + " of " + std::to_string(n) +
                                            " rows (" + std::to_string(at(n) - at(start)) + " more bytes needed)");
  return FORY_OK;
}

// Queues the D2H of rows [a, a + rows) (contiguous at `src`, row i at (i - a) * stride)
// into the windows they belong to.
int d2h_rows_windows(fory_host_ctx* c, const OutWindows& W, const uint8_t* src, int64_t a, int64_t rows, int64_t stride, hipStream_t s) {
  int rc = FORY_OK;
  for (size_t w = 0; w + 1 < W.first.size() && !rc; ++w) {
    const int64_t lo = std::max(a, W.first[w]), hi = std::min(a + rows, W.first[w + 1]);
    if (lo >= hi) continue;
    rc = hcopy(c, W.ptr[w] + (lo - W.first[w]) * stride, src + (lo - a) * stride, (size_t)((hi - lo) * stride), hipMemcpyDeviceToHost, s, "D2H");
  }
  return rc;
}

int host_encode_fixed(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame, OutWindows* W) {
  if (c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "varlen plan: use fory_rowfmt_host_encode_var");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM && frame != FORY_FRAME_HASHED)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "frame_mode must be 0 (raw), 1 (stream) or 3 (hashed)");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  const int64_t stride = c->info.fixed_size + (frame == FORY_FRAME_STREAM ? 12 : frame == FORY_FRAME_HASHED ? 8 : 0);
  int rc = split_rows(nullptr, stride, n, W);  // MemoryBuffer bounds check (MemoryBuffer.java:303-309)
  if (rc || n == 0) return rc;
  if (!host_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host columns are null");
  for (size_t w = 0; w + 1 < W->first.size(); ++w)
    if (W->first[w + 1] > W->first[w] && !W->ptr[w]) return fail_host(FORY_ERR_INVALID_ARGUMENT, "output is null");
  for (int i = 0; i < c->info.num_columns; ++i)
    if (!host_cols[i].values || host_cols[i].length < n)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " missing or shorter than num_rows");
  rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  for (int i = 0; i < c->info.num_columns; ++i) {
    call_extent(c, host_cols[i].values, n * c->width[i]);
    if (c->nullable[i]) call_extent(c, host_cols[i].validity, (n + 7) / 8);
  }
  for (size_t w = 0; w + 1 < W->first.size(); ++w)
    call_extent(c, W->ptr[w], (W->first[w + 1] - W->first[w]) * stride);
  for (int b = 0; b < 2 && !rc; ++b)
    rc = hip_check(hipMemsetAsync(c->buf[b].status, 0, 4, c->s_k), "hipMemsetAsync");
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  std::vector<fory_column> dcols(c->info.num_columns);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    int64_t a, rows;
    chunk_range(c, n, k, &a, &rows);
    fory_host_ctx::Buf& B = c->buf[b];
    // H2D: column slices (+ validity bytes) into buffer b once chunk k-2's kernel is done with it
    if (k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns && !rc; ++i) {
      const fory_column& h = host_cols[i];
      dcols[i] = fory_column{B.cols[i].values, nullptr, (c->nullable[i] && h.validity) ? B.cols[i].validity : nullptr,
                             rows, rows * c->width[i]};
      rc = hcopy(c, B.cols[i].values, static_cast<const uint8_t*>(h.values) + a * c->width[i], (size_t)(rows * c->width[i]), hipMemcpyHostToDevice, c->s_in, "H2D");
      if (!rc && c->nullable[i] && h.validity)
        rc = hcopy(c, B.cols[i].validity, h.validity + a / 8, (size_t)((rows + 7) / 8), hipMemcpyHostToDevice, c->s_in, "H2D validity");
    }
    if (!rc) rc = hip_check(hipEventRecord(c->ev_in[b], c->s_in), "hipEventRecord");
    if (!rc) rc = verify_pieces(c, c->s_in, k);
    // kernel: after the chunk landed and chunk k-2's rows left buffer b
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_in[b], 0), "hipStreamWaitEvent");
    if (!rc && k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_out[b], 0), "hipStreamWaitEvent");
    if (!rc)
      rc = fory_rowfmt_encode(c->plan, dcols.data(), rows, frame, nullptr, B.rows, rows * stride, B.status, B.ws,
                              c->ws_bytes, c->s_k);
    if (!rc) rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
    // D2H: the chunk's rows into the window(s) holding them
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
    if (!rc) rc = d2h_rows_windows(c, *W, B.rows, a, rows, stride, c->s_out);
    if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_out), "hipEventRecord");
  }
  const int rc_sync = sync_all(c);
  if (rc) return rc;
  if (rc_sync) return rc_sync;
  for (int b = 0; b < 2; ++b) {
    rc = fory_rowfmt_read_status(c->buf[b].status, c->s_k);
    if (rc) return rc;
  }
  return FORY_OK;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_encode(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                            void* host_out, int64_t out_capacity) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (n > 0 && !host_out) return fail_host(FORY_ERR_INVALID_ARGUMENT, "output is null");
  OutWindows W;
  W.ptr = {static_cast<uint8_t*>(host_out)};
  W.cap = {out_capacity};
  return host_encode_fixed(c, host_cols, n, frame, &W);
}

int fory_rowfmt_host_decode(fory_host_ctx* c, const void* host_rows, int64_t rows_bytes, int64_t n, int32_t frame,
                            const fory_column* host_out_cols) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "varlen plan: use fory_rowfmt_host_decode_var");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM && frame != FORY_FRAME_HASHED)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "frame_mode must be 0 (raw), 1 (stream) or 3 (hashed)");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (n == 0) return FORY_OK;
  if (!host_rows || !host_out_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows or output columns null");
  const int64_t stride = c->info.fixed_size + (frame == FORY_FRAME_STREAM ? 12 : frame == FORY_FRAME_HASHED ? 8 : 0);
  if (n * stride > rows_bytes)
    return fail_host(FORY_ERR_CORRUPT, "row buffer holds " + std::to_string(rows_bytes) + " bytes < " +
                                           std::to_string(n) + " rows x " + std::to_string(stride));
  for (int i = 0; i < c->info.num_columns; ++i) {
    const fory_column& h = host_out_cols[i];
    if (!h.values || (h.capacity > 0 && h.capacity < n * c->width[i]))
      return fail_host(FORY_ERR_CAPACITY, "output column " + std::to_string(i) + " missing or too small");
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  // in the order the copies first need them: the first chunk's rows, the output columns
  // (its D2H), then the other chunks' rows
  const int64_t first = std::min(n, c->chunk) * stride;
  call_extent(c, host_rows, first);
  for (int i = 0; i < c->info.num_columns; ++i) {
    call_extent(c, host_out_cols[i].values, n * c->width[i]);
    if (c->nullable[i]) call_extent(c, host_out_cols[i].validity, (n + 7) / 8);
  }
  call_extent(c, static_cast<const uint8_t*>(host_rows) + first, n * stride - first);
  for (int b = 0; b < 2 && !rc; ++b)
    rc = hip_check(hipMemsetAsync(c->buf[b].status, 0, 4, c->s_k), "hipMemsetAsync");
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  std::vector<fory_column> dcols(c->info.num_columns);
  const uint8_t* in = static_cast<const uint8_t*>(host_rows);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    int64_t a, rows;
    chunk_range(c, n, k, &a, &rows);
    fory_host_ctx::Buf& B = c->buf[b];
    if (k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");
    if (!rc)
      rc = hcopy(c, B.rows, in + a * stride, (size_t)(rows * stride), hipMemcpyHostToDevice, c->s_in, "H2D");
    if (!rc) rc = hip_check(hipEventRecord(c->ev_in[b], c->s_in), "hipEventRecord");
    if (!rc) rc = verify_pieces(c, c->s_in, k);
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_in[b], 0), "hipStreamWaitEvent");
    if (!rc && k >= 2) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_out[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns; ++i)
      dcols[i] = fory_column{B.cols[i].values, nullptr,
                             (c->nullable[i] && host_out_cols[i].validity) ? B.cols[i].validity : nullptr, rows,
                             rows * c->width[i]};
    if (!rc) rc = fory_rowfmt_decode(c->plan, B.rows, nullptr, rows, frame, dcols.data(), B.status, B.ws, c->ws_bytes,
                                     c->s_k);
    if (!rc) rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
    for (int i = 0; i < c->info.num_columns && !rc; ++i) {
      const fory_column& h = host_out_cols[i];
      rc = hcopy(c, static_cast<uint8_t*>(h.values) + a * c->width[i], B.cols[i].values, (size_t)(rows * c->width[i]), hipMemcpyDeviceToHost, c->s_out, "D2H");
      if (!rc && dcols[i].validity)
        rc = hcopy(c, h.validity + a / 8, B.cols[i].validity, (size_t)((rows + 7) / 8), hipMemcpyDeviceToHost, c->s_out, "D2H validity");
    }
    if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_out), "hipEventRecord");
  }
  const int rc_sync = sync_all(c);
  if (rc) return rc;
  if (rc_sync) return rc_sync;
  for (int b = 0; b < 2; ++b) {
    rc = fory_rowfmt_read_status(c->buf[b].status, c->s_k);
    if (rc) return rc;
  }
  return FORY_OK;
}


// ---------------------------------------------------------------------------
// Varlen plans (strings, lists, maps, nested structs, collection frames): the
// whole batch per call. Row sizes are data-dependent, so the chunk pipeline's
// fixed strides do not apply; device buffers live in the context and grow.
// ---------------------------------------------------------------------------

}  // extern "C"

namespace {

constexpr int32_t kKindFixed = 0, kKindBool = 1, kKindBytes = 2, kKindStruct = 3, kKindList = 4, kKindMap = 5;

bool has_offsets(int32_t k) { return k == kKindBytes || k == kKindList || k == kKindMap; }

// Grows a context-owned device buffer (synchronising the context's stream first).
// Regrowing dbuf or drows frees what a staged decode (host_decode_var_sizes ->
// host_decode_var) points into, so it also drops that staged state.
int ensure(fory_host_ctx* c, uint8_t** buf, int64_t* have, int64_t need) {
  if (need <= *have) return FORY_OK;
  if (buf == &c->dbuf || buf == &c->drows) c->dec_n = -1;
  int rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
  if (rc) return rc;
  if (*buf) (void)hipFree(*buf);
  *buf = nullptr;
  *have = 0;
  const int64_t sz = align_up(need + need / 4);
  rc = hip_check(hipMalloc(buf, (size_t)sz), "hipMalloc(host ctx varlen buffers)");
  if (!rc) *have = sz;
  return rc;
}

// Carves per-column device regions (values, offsets, validity) for the element
// counts / value bytes given, then row offsets (n+1 int64), the workspace and the
// status word; returns the bytes needed when base is null.
int64_t carve(fory_host_ctx* c, uint8_t* base, const std::vector<int64_t>& cnt, const std::vector<int64_t>& vbytes,
              const std::vector<char>& want_validity, int64_t n, std::vector<fory_column>* cols, int64_t** d_offs,
              void** ws, int64_t ws_bytes, int32_t** status) {
  int64_t at = 0;
  const int N = (int)cnt.size();
  if (cols) cols->assign(N, fory_column{});
  for (int i = 0; i < N; ++i) {
    fory_column d{};
    d.length = cnt[i];
    if (vbytes[i] > 0 || c->kind[i] == kKindFixed || c->kind[i] == kKindBool || c->kind[i] == kKindBytes) {
      d.values = base ? base + at : nullptr;
      d.capacity = vbytes[i];
      at += align_up(vbytes[i] > 0 ? vbytes[i] : 1);
    }
    if (has_offsets(c->kind[i]) && cnt[i] >= 0) {
      d.offsets = base ? reinterpret_cast<int32_t*>(base + at) : nullptr;
      at += align_up((cnt[i] + 1) * 4);
    }
    if (want_validity[i]) {
      d.validity = base ? base + at : nullptr;
      at += align_up(validity_bytes(cnt[i] > 0 ? cnt[i] : 1));
    }
    if (cols) (*cols)[i] = d;
  }
  if (d_offs) *d_offs = base ? reinterpret_cast<int64_t*>(base + at) : nullptr;
  at += align_up((n + 1) * 8);
  if (ws) *ws = base ? base + at : nullptr;
  at += align_up(ws_bytes);
  if (status) *status = base ? reinterpret_cast<int32_t*>(base + at) : nullptr;
  at += kAlign;
  return at;
}

}  // namespace

namespace {

// Chunk k's slice of a varlen batch (rows [a, a + rows)) per pre-order column:
// elements [lo, hi) are the chunk's own — the rows themselves at the top level and in
// struct fields, below a list/map the children its offsets name. The H2D copies
// start at aligned host positions and the device column pointers are biased back
// ("virtual bases"): the kernels index a slice with the host's absolute element
// indices and offsets (top level: chunk-row indices), so nothing is rebased.
struct VarSlice {
  int64_t lo = 0, hi = 0;  // absolute element range
  int64_t s = 0;           // absolute element the kernels' index 0 denotes (a at the top, 0 below a list/map)
  int64_t v0 = 0, v1 = 0;  // host value bytes copied (v0 16-byte aligned)
  int64_t o0 = 0;          // first offsets entry copied (a multiple of 4), through entry hi
  int64_t h0 = 0, h1 = 0;  // host validity bytes copied (h0 a multiple of 8)
  bool validity = false;
};

constexpr int64_t kSlack = 64;  // the kernels' aligned loads may read past a span's end

int var_slices(const fory_host_ctx* c, const fory_column* h, int64_t a, int64_t rows, std::vector<VarSlice>* out) {
  const int N = c->info.num_columns;
  out->assign((size_t)N, VarSlice{});
  for (int i = 0; i < N; ++i) {
    VarSlice& v = (*out)[(size_t)i];
    const int p = c->parent[i];
    if (p < 0) {
      v.lo = a, v.hi = a + rows, v.s = a;
    } else if (c->kind[p] == kKindStruct) {
      v.lo = (*out)[(size_t)p].lo, v.hi = (*out)[(size_t)p].hi, v.s = (*out)[(size_t)p].s;
    } else {  // list items / map entries of the chunk
      v.lo = h[p].offsets[(*out)[(size_t)p].lo];
      v.hi = h[p].offsets[(*out)[(size_t)p].hi];
      v.s = 0;
      if (v.lo < 0 || v.hi < v.lo) return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(p) + " offsets decrease");
    }
    if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) {
      v.v0 = (v.lo * c->width[i]) & ~int64_t(15);
      v.v1 = v.hi * c->width[i];
    } else if (c->kind[i] == kKindBytes) {
      const int64_t b0 = h[i].offsets[v.lo], b1 = h[i].offsets[v.hi];
      if (b0 < 0 || b1 < b0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " offsets decrease");
      v.v0 = b0 & ~int64_t(15);
      v.v1 = b1;
    }
    if (v.v1 > v.v0 && !h[i].values)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " has no values");
    v.o0 = v.lo & ~int64_t(3);
    v.validity = c->nullable[i] && h[i].validity;
    if (v.validity) {
      v.h0 = (v.lo >> 3) & ~int64_t(7);
      v.h1 = (v.hi + 7) >> 3;
    }
  }
  return FORY_OK;
}

// Bytes of a slot's device region for these slices (base null), or carves it: the
// biased device columns, the chunk's row offsets and the workspace.
int64_t carve_slices(const fory_host_ctx* c, const std::vector<VarSlice>& sl, int64_t rows, int64_t ws_bytes,
                     uint8_t* base, std::vector<fory_column>* cols, int64_t** d_offs, void** ws) {
  int64_t at = 0;
  const int N = (int)sl.size();
  if (cols) cols->assign((size_t)N, fory_column{});
  for (int i = 0; i < N; ++i) {
    const VarSlice& v = sl[(size_t)i];
    fory_column d{};
    d.length = v.hi - v.lo;
    if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool || c->kind[i] == kKindBytes) {
      const int64_t bias = c->kind[i] == kKindBytes ? -v.v0 : v.s * c->width[i] - v.v0;
      if (base) d.values = base + at + bias;
      d.capacity = v.v1 - v.v0;
      at += align_up(v.v1 - v.v0 + kSlack);
    }
    if (has_offsets(c->kind[i])) {
      if (base) d.offsets = reinterpret_cast<int32_t*>(base + at) + (v.s - v.o0);
      at += align_up((v.hi - v.o0 + 1) * 4 + kSlack);
    }
    if (v.validity) {
      if (base) d.validity = base + at + ((v.s >> 3) - v.h0);
      at += align_up(v.h1 - v.h0 + kSlack);
    }
    if (cols) (*cols)[(size_t)i] = d;
  }
  if (d_offs) *d_offs = base ? reinterpret_cast<int64_t*>(base + at) : nullptr;
  at += align_up((rows + 1) * 8);
  if (ws) *ws = base ? base + at : nullptr;
  at += align_up(ws_bytes);
  return at;
}

// The caller's columns of a varlen call as call extents (values, offsets, validity of
// each pre-order column; a column's length is its element count).
void declare_column_extents(fory_host_ctx* c, const fory_column* h) {
  for (int i = 0; i < c->info.num_columns; ++i) {
    const int64_t len = h[i].length;
    if (len <= 0) continue;
    if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) call_extent(c, h[i].values, len * c->width[i]);
    if (c->kind[i] == kKindBytes && h[i].offsets) call_extent(c, h[i].values, h[i].offsets[len]);
    if (has_offsets(c->kind[i])) call_extent(c, h[i].offsets, (len + 1) * 4);
    if (c->nullable[i]) call_extent(c, h[i].validity, (len + 7) / 8);
  }
}

// H2D of the slices into a slot's carved region (the unbiased region starts).
int h2d_slices(fory_host_ctx* c, const fory_column* h, const std::vector<VarSlice>& sl,
               const std::vector<fory_column>& d, hipStream_t s) {
  int rc = FORY_OK;
  for (size_t i = 0; i < sl.size() && !rc; ++i) {
    const VarSlice& v = sl[i];
    if (d[i].values && v.v1 > v.v0) {
      const int64_t bias = c->kind[i] == kKindBytes ? -v.v0 : v.s * c->width[i] - v.v0;
      rc = hcopy(c, static_cast<uint8_t*>(d[i].values) - bias, static_cast<const uint8_t*>(h[i].values) + v.v0,
                 (size_t)(v.v1 - v.v0), hipMemcpyHostToDevice, s, "H2D values");
    }
    if (!rc && d[i].offsets)
      rc = hcopy(c, d[i].offsets - (v.s - v.o0), h[i].offsets + v.o0, (size_t)(v.hi - v.o0 + 1) * 4,
                 hipMemcpyHostToDevice, s, "H2D offsets");
    if (!rc && v.validity && v.h1 > v.h0)
      rc = hcopy(c, d[i].validity - ((v.s >> 3) - v.h0), h[i].validity + v.h0, (size_t)(v.h1 - v.h0),
                 hipMemcpyHostToDevice, s, "H2D validity");
  }
  return rc;
}

// Varlen encode, chunk pipeline over two slots. Per chunk k (slot b = k & 1):
//   s_in : H2D of its column slices -> encoded_size (row sizes + scan) -> D2H of its
//          row offsets to pinned memory (ev_sz)
//   host : waits for ev_sz, places the chunk after the rows so far (windows, output
//          row offsets), grows the slot's row buffer if needed
//   s_k  : encode into the slot's row buffer (ev_k)
//   s_out: D2H of the rows into their window(s) (ev_out)
// Chunk k+1 is staged before chunk k's encode is queued, so H2D (k+1) || encode (k)
// || D2H (k-1). A window overflow stops the copies; the remaining chunks are only
// sized, so *out_bytes reports the total (then FORY_ERR_CAPACITY).
int host_encode_var(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame, OutWindows* W,
                    int64_t* host_row_offsets, int64_t* out_bytes) {
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_encode");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (out_bytes) *out_bytes = 0;
  const int64_t nw = (int64_t)W->cap.size();
  if (n == 0) {
    if (host_row_offsets) host_row_offsets[0] = 0;
    W->first.assign((size_t)nw + 1, 0);
    return FORY_OK;
  }
  if (!host_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host columns are null");
  // a context serves one call at a time: a staged decode does not survive an encode
  c->dec_n = -1;
  const int N = c->info.num_columns;
  for (int i = 0; i < N; ++i)
    if (has_offsets(c->kind[i]) && !host_cols[i].offsets)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(i) + " needs offsets");
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  declare_column_extents(c, host_cols);
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, std::min(n, c->chunk));
  rc = hip_check(hipMemsetAsync(c->vstatus, 0, 8, c->s_k), "hipMemsetAsync");
  if (!rc) rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
  if (rc) return rc;
  std::vector<fory_column> dcols[2];
  int64_t* d_offs[2] = {};
  void* ws[2] = {};
  int64_t crow[2] = {}, c0[2] = {};  // rows and first row of the chunk in each slot

  // H2D + sizes of chunk k into slot k & 1 (queued on s_in)
  auto stage = [&](int64_t k) -> int {
    const int b = (int)(k & 1);
    fory_host_ctx::VarSlot& S = c->vs[b];
    const int64_t a = k * c->chunk, rows = std::min(c->chunk, n - a);
    std::vector<VarSlice> sl;
    int r = var_slices(c, host_cols, a, rows, &sl);
    if (r) return r;
    const int64_t need = carve_slices(c, sl, rows, ws_bytes, nullptr, nullptr, nullptr, nullptr);
    if (S.used) r = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");  // chunk k-2 read it
    if (!r && need > S.dev_bytes) {
      if (S.used) r = hip_check(hipEventSynchronize(c->ev_k[b]), "hipEventSynchronize");
      if (S.dev) (void)hipFree(S.dev);
      S.dev = nullptr, S.dev_bytes = 0;
      const int64_t sz = align_up(need + need / 4);
      if (!r) r = hip_check(hipMalloc(&S.dev, (size_t)sz), "hipMalloc(host ctx chunk slot)");
      if (!r) S.dev_bytes = sz;
    }
    if (!r && S.pin_words < rows + 1) {
      if (S.used) r = hip_check(hipEventSynchronize(c->ev_sz[b]), "hipEventSynchronize");
      if (S.pin) (void)hipHostFree(S.pin);
      S.pin = nullptr, S.pin_words = 0;
      if (!r) r = hip_check(hipHostMalloc(reinterpret_cast<void**>(&S.pin), (size_t)(c->chunk + 1) * 8, hipHostMallocCoherent),
                            "hipHostMalloc(row offsets)");
      if (!r) S.pin_words = c->chunk + 1;
    }
    if (r) return r;
    carve_slices(c, sl, rows, ws_bytes, S.dev, &dcols[b], &d_offs[b], &ws[b]);
    r = h2d_slices(c, host_cols, sl, dcols[b], c->s_in);
    if (!r) r = verify_pieces(c, c->s_in, k);
    if (!r) r = fory_rowfmt_encoded_size(c->plan, dcols[b].data(), rows, frame, d_offs[b], ws[b], ws_bytes, c->s_in);
    if (!r) r = hcopy(c, S.pin, d_offs[b], (size_t)(rows + 1) * 8, hipMemcpyDeviceToHost, c->s_in, "D2H row offsets");
    if (!r) r = hip_check(hipEventRecord(c->ev_sz[b], c->s_in), "hipEventRecord");
    crow[b] = rows, c0[b] = a;
    return r;
  };

  // greedy window placement (split_rows, incrementally): window w started at row
  // first[w]; its byte limit is that row's offset + cap[w]
  W->first.assign((size_t)nw + 1, n);
  std::vector<int64_t> wbyte((size_t)nw + 1, 0);  // batch byte offset where window w starts
  int64_t w = 0, wlimit = W->cap.empty() ? -1 : W->cap[0];
  W->first[0] = 0;
  bool overflow = nw == 0;
  int64_t base = 0;  // bytes of the chunks before
  rc = stage(0);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    fory_host_ctx::VarSlot& S = c->vs[b];
    if (k + 1 < chunks) rc = stage(k + 1);
    if (!rc) rc = hip_check(hipEventSynchronize(c->ev_sz[b]), "hipEventSynchronize");
    if (rc) break;
    const int64_t a = c0[b], rows = crow[b];
    const int64_t* po = S.pin;
    const int64_t total = po[rows];
    if (host_row_offsets)
      for (int64_t i = 0; i <= rows; ++i) host_row_offsets[a + i] = base + po[i];
    // rows of this chunk per window: [lo, hi) of the batch
    auto at = [&](int64_t e) { return base + po[e - a]; };
    std::vector<int64_t> piece_w, piece_lo, piece_hi;
    int64_t cur = a;
    while (!overflow && cur < a + rows) {
      int64_t lo = cur, hi = a + rows;  // largest e in [cur, a + rows] with at(e) <= wlimit
      while (lo < hi) {
        const int64_t mid = hi - (hi - lo) / 2;
        if (at(mid) <= wlimit) lo = mid;
        else hi = mid - 1;
      }
      if (lo > cur) piece_w.push_back(w), piece_lo.push_back(cur), piece_hi.push_back(lo);
      cur = lo;
      if (cur < a + rows) {  // row cur does not fit window w: the next window starts there
        W->first[(size_t)++w] = cur;
        wbyte[(size_t)w] = at(cur);
        if (w == nw) overflow = true;
        else wlimit = at(cur) + W->cap[(size_t)w];
      }
    }
    for (int64_t pw : piece_w)
      if (!W->ptr[(size_t)pw]) rc = fail_host(FORY_ERR_INVALID_ARGUMENT, "output is null");
    if (!overflow && !rc) {
      if (S.used) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_out[b], 0), "hipStreamWaitEvent");  // k-2's D2H
      if (!rc && total + 16 > S.rows_bytes) {
        if (S.used) rc = hip_check(hipEventSynchronize(c->ev_out[b]), "hipEventSynchronize");
        if (S.rows) (void)hipFree(S.rows);
        S.rows = nullptr, S.rows_bytes = 0;
        const int64_t sz = align_up(total + total / 4 + 16);
        if (!rc) rc = hip_check(hipMalloc(&S.rows, (size_t)sz), "hipMalloc(host ctx chunk rows)");
        if (!rc) S.rows_bytes = sz;
      }
      if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_sz[b], 0), "hipStreamWaitEvent");
      if (!rc)
        rc = fory_rowfmt_encode(c->plan, dcols[b].data(), rows, frame, d_offs[b], S.rows, total, c->vstatus + b,
                                ws[b], ws_bytes, c->s_k);
      if (!rc) rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
      if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
      for (size_t q = 0; q < piece_w.size(); ++q)  // this chunk's output pieces: registered as they are copied
        call_extent(c, W->ptr[(size_t)piece_w[q]] + (at(piece_lo[q]) - wbyte[(size_t)piece_w[q]]),
                    at(piece_hi[q]) - at(piece_lo[q]));
      for (size_t q = 0; q < piece_w.size() && !rc; ++q) {
        const int64_t pw = piece_w[q];
        rc = hcopy(c, W->ptr[(size_t)pw] + (at(piece_lo[q]) - wbyte[(size_t)pw]), S.rows + po[piece_lo[q] - a], (size_t)(at(piece_hi[q]) - at(piece_lo[q])), hipMemcpyDeviceToHost,
                   c->s_out, "D2H rows");
      }
      if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_out), "hipEventRecord");
    } else if (!rc) {  // sizes only from here: the slot's columns are free again once sized
      rc = hip_check(hipEventRecord(c->ev_k[b], c->s_in), "hipEventRecord");
      if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_in), "hipEventRecord");
    }
    S.used = true;
    base += total;
  }
  const int rc_sync = sync_all(c);
  if (rc) return rc;
  if (rc_sync) return rc_sync;
  if (out_bytes) *out_bytes = base;
  if (overflow) {
    int64_t placed = nw > 0 ? W->first[(size_t)nw] : 0;
    return fail_host(FORY_ERR_CAPACITY, "output windows hold " + std::to_string(placed) + " of " + std::to_string(n) +
                                            " rows (" + std::to_string(base) + " bytes in all)");
  }
  for (int b = 0; b < 2 && !rc; ++b) rc = fory_rowfmt_read_status(c->vstatus + b, c->s_k);
  return rc;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_encode_var(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                                void* host_out, int64_t out_capacity, int64_t* host_row_offsets,
                                int64_t* out_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  OutWindows W;
  W.ptr = {static_cast<uint8_t*>(host_out)};
  W.cap = {out_capacity};
  return host_encode_var(c, host_cols, n, frame, &W, host_row_offsets, out_bytes);
}

int fory_rowfmt_host_encode_windows(fory_host_ctx* c, const fory_column* host_cols, int64_t n, int32_t frame,
                                    void* const* windows, const int64_t* window_caps, int32_t num_windows,
                                    int64_t* window_rows, int64_t* window_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (num_windows <= 0 || !windows || !window_caps)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "windows / window_caps null or num_windows <= 0");
  OutWindows W;
  for (int32_t w = 0; w < num_windows; ++w) {
    if (window_caps[w] < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "window capacity < 0");
    W.ptr.push_back(static_cast<uint8_t*>(windows[w]));
    W.cap.push_back(window_caps[w]);
  }
  int rc;
  int64_t stride = 0;
  std::vector<int64_t> offs;
  if (c->varlen) {
    offs.resize((size_t)(n > 0 ? n : 0) + 1, 0);
    rc = host_encode_var(c, host_cols, n, frame, &W, offs.data(), nullptr);
  } else {
    stride = c->info.fixed_size + (frame == FORY_FRAME_STREAM ? 12 : frame == FORY_FRAME_HASHED ? 8 : 0);
    rc = host_encode_fixed(c, host_cols, n, frame, &W);
  }
  if (rc) return rc;
  if (W.first.size() != (size_t)num_windows + 1) W.first.assign((size_t)num_windows + 1, 0);
  for (int32_t w = 0; w < num_windows; ++w) {
    const int64_t f0 = W.first[(size_t)w], f1 = W.first[(size_t)w + 1];
    if (window_rows) window_rows[w] = f1 - f0;
    if (window_bytes) window_bytes[w] = c->varlen ? offs[(size_t)f1] - offs[(size_t)f0] : (f1 - f0) * stride;
  }
  return FORY_OK;
}

}  // extern "C"

namespace {

// Stages a decode batch on the device: rows (host_row_offsets given: the run
// [offs[0], offs[n]) with offsets rebased to it; else the first rows_bytes bytes of
// a frame stream, indexed on the device by fory_rowfmt_index_frames) and sizes
// every output column (fory_rowfmt_decode_sizes, repeated while list/map element
// counts become known). The staged state serves the next host_decode_var.
int decode_var_stage(fory_host_ctx* c, const void* host_rows, const int64_t* host_row_offsets, int64_t rows_bytes,
                     int64_t n, int32_t frame, int64_t* host_counts, int64_t* host_bytes, int64_t* consumed) {
  const int N = c->info.num_columns;
  c->dec_n = -1;
  int64_t r0 = 0, r1 = rows_bytes;
  if (host_row_offsets) {
    r0 = host_row_offsets[0];
    r1 = host_row_offsets[n];
    if (r1 < r0 || r0 < 0) return fail_host(FORY_ERR_CORRUPT, "row offsets decrease");
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  call_extent(c, static_cast<const uint8_t*>(host_rows) + r0, r1 - r0);
  // device run: [rows (16-byte aligned start)][row offsets n+1][index status][index workspace]
  const int64_t rows_sz = align_up((r1 - r0) + 16), offs_sz = align_up((n + 1) * 8);
  const int64_t iws = host_row_offsets ? 0 : fory_rowfmt_index_workspace_bytes(c->plan, n, r1 - r0);
  rc = ensure(c, &c->drows, &c->drows_bytes, rows_sz + offs_sz + kAlign + iws);
  if (!rc) rc = ensure_hpin(c, 16 + 4 * (int64_t)N);
  if (rc) return rc;
  uint8_t* drow0 = c->drows;
  int64_t* d_offs = reinterpret_cast<int64_t*>(c->drows + rows_sz);
  int32_t* istatus = reinterpret_cast<int32_t*>(c->drows + rows_sz + offs_sz);
  if (r1 > r0)
    rc = hcopy(c, drow0, static_cast<const uint8_t*>(host_rows) + r0, (size_t)(r1 - r0), hipMemcpyHostToDevice, c->s_k, "H2D rows");
  if (host_row_offsets) {  // row offsets relative to the staged run
    std::vector<int64_t> rel_offs((size_t)n + 1);
    for (int64_t k = 0; k <= n; ++k) rel_offs[(size_t)k] = host_row_offsets[k] - r0;
    if (!rc)
      rc = hcopy(c, d_offs, rel_offs.data(), (size_t)(n + 1) * 8, hipMemcpyHostToDevice, c->s_k, "H2D row offsets");
    if (consumed) *consumed = r1;  // (rel_offs is staged: pinned before hcopy returns)
  } else {  // Encoder.decode(MemoryBuffer) x n over the stream alone
    if (!rc) rc = hip_check(hipMemsetAsync(istatus, 0, 4, c->s_k), "hipMemsetAsync");
    if (!rc)
      rc = fory_rowfmt_index_frames(c->plan, drow0, r1 - r0, n, frame, d_offs, istatus,
                                    c->drows + rows_sz + offs_sz + kAlign, iws, c->s_k);
    int64_t* end = reinterpret_cast<int64_t*>(c->hpin);  // pinned: an async D2H, read after the sync
    if (!rc) rc = hip_check(hipMemcpyAsync(end, d_offs + n, 8, hipMemcpyDeviceToHost, c->s_k), "D2H frame end");
    if (!rc) rc = fory_rowfmt_read_status(istatus, c->s_k);  // synchronises the stream
    if (rc) return rc;
    if (consumed) *consumed = *end;
  }
  if (rc) return rc;
  // element counts: top level n; struct fields as their struct; list/map elements
  // from the container totals (pass 1), string/binary elements' bytes (pass 2)
  std::vector<int64_t> cnt(N, -1), vbytes(N, 0);
  std::vector<char> want_validity(N, 0);
  for (int i = 0; i < N; ++i) want_validity[i] = c->nullable[i] != 0;
  auto resolve = [&]() {
    for (int i = 0; i < N; ++i) {
      const int p = c->parent[i];
      if (cnt[i] >= 0) continue;
      if (p < 0) cnt[i] = n;
      else if (cnt[p] >= 0 && c->kind[p] == kKindStruct) cnt[i] = cnt[p];
    }
  };
  resolve();
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, n);
  std::vector<fory_column> d;
  void* ws = nullptr;
  int32_t* status = nullptr;
  for (int pass = 0; pass < 20 && !rc; ++pass) {  // one level of list/map nesting per pass (<= 17)
    // layout for the counts known so far (unknown: no buffers, length 0)
    std::vector<int64_t> kc(N);
    for (int i = 0; i < N; ++i) kc[i] = cnt[i] < 0 ? -1 : cnt[i];
    std::vector<int64_t> vb0(N, 0);
    std::vector<char> wv(N, 0);
    rc = ensure(c, &c->dbuf, &c->dbuf_bytes, carve(c, nullptr, kc, vb0, wv, n, nullptr, nullptr, nullptr, ws_bytes,
                                                   nullptr));
    if (rc) break;
    carve(c, c->dbuf, kc, vb0, wv, n, &d, nullptr, &ws, ws_bytes, &status);
    for (int i = 0; i < N; ++i) {
      d[i].values = nullptr;
      d[i].capacity = 0;
      if (kc[i] < 0) d[i] = fory_column{};
    }
    rc = hip_check(hipMemsetAsync(status, 0, 4, c->s_k), "hipMemsetAsync");
    if (!rc)
      rc = fory_rowfmt_decode_sizes(c->plan, drow0, d_offs, n, frame, d.data(), status, ws, ws_bytes, c->s_k);
    int32_t* tot = reinterpret_cast<int32_t*>(c->hpin + 16);  // pinned level totals
    for (int i = 0; i < N; ++i) tot[i] = 0;
    for (int i = 0; i < N && !rc; ++i)
      if (d[i].offsets && kc[i] >= 0)
        rc = hip_check(hipMemcpyAsync(&tot[i], d[i].offsets + kc[i], 4, hipMemcpyDeviceToHost, c->s_k), "D2H totals");
    if (!rc) rc = fory_rowfmt_read_status(status, c->s_k);  // synchronises the stream
    if (rc) break;
    bool changed = false;
    for (int i = 0; i < N; ++i) {
      if (!has_offsets(c->kind[i]) || kc[i] < 0) continue;
      if (c->kind[i] == kKindBytes) vbytes[i] = tot[i];
      else
        for (int j = 0; j < N; ++j)  // direct children of a list/map: its element total
          if (c->parent[j] == i && cnt[j] < 0) cnt[j] = tot[i], changed = true;
    }
    resolve();
    if (!changed) break;
  }
  if (rc) return rc;
  for (int i = 0; i < N; ++i) {
    if (cnt[i] < 0) cnt[i] = 0;
    if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) vbytes[i] = cnt[i] * c->width[i];
    host_counts[i] = cnt[i];
    host_bytes[i] = vbytes[i];
  }
  c->dec_n = n;
  c->dec_frame = frame;
  c->dec_count = cnt;
  c->dec_bytes = vbytes;
  c->dec_cols = d;  // the last pass's device offsets (tile bases / totals for decode)
  c->dec_offs = d_offs;  // in the drows run
  c->dec_ws = ws;
  c->dec_status = status;
  return FORY_OK;
}

}  // namespace

extern "C" {

int fory_rowfmt_host_decode_var_sizes(fory_host_ctx* c, const void* host_rows, const int64_t* host_row_offsets,
                                      int64_t n, int32_t frame, int64_t* host_counts, int64_t* host_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_decode");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (!host_row_offsets || !host_counts || !host_bytes || (n > 0 && !host_rows))
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows, row offsets or size outputs null");
  return decode_var_stage(c, host_rows, host_row_offsets, 0, n, frame, host_counts, host_bytes, nullptr);
}

int fory_rowfmt_host_decode_stream_sizes(fory_host_ctx* c, const void* host_rows, int64_t rows_bytes, int64_t n,
                                         int64_t* host_counts, int64_t* host_bytes, int64_t* consumed_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_decode");
  if (n < 0 || rows_bytes < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows or rows_bytes < 0");
  if (!host_counts || !host_bytes || (n > 0 && !host_rows))
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows or size outputs null");
  return decode_var_stage(c, host_rows, nullptr, rows_bytes, n, FORY_FRAME_STREAM, host_counts, host_bytes,
                          consumed_bytes);
}

int fory_rowfmt_host_decode_var(fory_host_ctx* c, const fory_column* host_out_cols) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen || c->dec_n < 0)
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "call fory_rowfmt_host_decode_var_sizes first");
  const int N = c->info.num_columns;
  const int64_t n = c->dec_n;
  if (n > 0 && !host_out_cols) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host output columns null");
  for (int i = 0; i < N && n > 0; ++i) {
    const fory_column& h = host_out_cols[i];
    if (c->dec_bytes[i] > 0 && (!h.values || (h.capacity > 0 && h.capacity < c->dec_bytes[i])))
      return fail_host(FORY_ERR_CAPACITY, "output column " + std::to_string(i) + " values missing or too small");
    if (has_offsets(c->kind[i]) && !h.offsets)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "output column " + std::to_string(i) + " needs offsets");
  }
  if (n == 0) {
    for (int i = 0; i < N; ++i)
      if (host_out_cols && host_out_cols[i].offsets) host_out_cols[i].offsets[0] = 0;
    return FORY_OK;
  }
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  for (int i = 0; i < N; ++i) {
    const fory_column& h = host_out_cols[i];
    call_extent(c, h.values, c->dec_bytes[i]);
    if (has_offsets(c->kind[i])) call_extent(c, h.offsets, (c->dec_count[i] + 1) * 4);
    if (c->nullable[i]) call_extent(c, h.validity, (c->dec_count[i] + 7) / 8);
  }
  std::vector<char> wv(N, 0);
  for (int i = 0; i < N; ++i) wv[i] = c->nullable[i] && host_out_cols[i].validity;
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, n);
  // output columns in their own buffer (the row offsets / workspace stay in dbuf)
  rc = ensure(c, &c->dout, &c->dout_bytes, carve(c, nullptr, c->dec_count, c->dec_bytes, wv, 0, nullptr, nullptr,
                                                 nullptr, 0, nullptr));
  if (rc) return rc;
  std::vector<fory_column> d;
  carve(c, c->dout, c->dec_count, c->dec_bytes, wv, 0, &d, nullptr, nullptr, 0, nullptr);
  const std::vector<int64_t>& kc = c->dec_count;
  const std::vector<fory_column>& dsz = c->dec_cols;
  int64_t* d_offs = c->dec_offs;
  void* ws = c->dec_ws;
  int32_t* status = c->dec_status;
  // the sizes pass wrote the offsets into dbuf's column regions: copy them over
  for (int i = 0; i < N && !rc; ++i) {
    if (d[i].offsets && dsz[i].offsets)
      rc = hip_check(hipMemcpyAsync(d[i].offsets, dsz[i].offsets, (size_t)(kc[i] + 1) * 4, hipMemcpyDeviceToDevice,
                                    c->s_k), "D2D offsets");
    if (!rc && d[i].validity)
      rc = hip_check(hipMemsetAsync(d[i].validity, 0, (size_t)validity_bytes(kc[i] > 0 ? kc[i] : 1), c->s_k),
                     "hipMemsetAsync");
  }
  if (!rc) rc = hip_check(hipMemsetAsync(status, 0, 4, c->s_k), "hipMemsetAsync");
  if (!rc)
    rc = fory_rowfmt_decode(c->plan, c->drows, d_offs, n, c->dec_frame, d.data(), status, ws, ws_bytes, c->s_k);
  for (int i = 0; i < N && !rc; ++i) {  // D2H of every column
    const fory_column& h = host_out_cols[i];
    if (d[i].values && c->dec_bytes[i] > 0)
      rc = hcopy(c, h.values, d[i].values, (size_t)c->dec_bytes[i], hipMemcpyDeviceToHost, c->s_k, "D2H values");
    if (!rc && d[i].offsets)
      rc = hcopy(c, h.offsets, d[i].offsets, (size_t)(kc[i] + 1) * 4, hipMemcpyDeviceToHost, c->s_k, "D2H offsets");
    if (!rc && d[i].validity)
      rc = hcopy(c, h.validity, d[i].validity, (size_t)((kc[i] + 7) / 8), hipMemcpyDeviceToHost, c->s_k, "D2H validity");
  }
  if (!rc) rc = fory_rowfmt_read_status(status, c->s_k);
  const int rd = stage_drain(c->stage);  // staged D2H pieces into the caller's columns
  return rc ? rc : rd;
}

}  // extern "C"

namespace {

// One-call varlen decode, chunk pipeline over the two slots. Per chunk k (slot b):
//   s_in : H2D of its row run and chunk-relative row offsets (queued one chunk ahead)
//   s_k  : decode_sizes, once per list/map level (the host reads each level's totals),
//          then the values pass into the slot's output region; offsets moved by the
//          elements of the chunks before, validity bits shifted to their batch bit
//   s_out: D2H of every column slice to its place in the caller's columns
// so H2D (k+1) || sizes + decode (k) || D2H (k-1). A validity byte shared by two
// chunks is written whole by the chunk holding its bit 0 and OR-ed by the other
// (from a pinned stash, after the last copy). Columns that would overflow the
// caller's capacities stop the copies; the rest of the batch is only sized.
int host_decode_var_into(fory_host_ctx* c, const uint8_t* host_rows, const int64_t* host_row_offsets, int64_t n,
                         int32_t frame, const fory_column* out, int64_t* host_counts, int64_t* host_bytes) {
  const int N = c->info.num_columns;
  c->dec_n = -1;  // a staged two-call decode does not survive this call
  for (int i = 0; i < N; ++i) host_counts[i] = 0, host_bytes[i] = 0;
  if (n == 0) {
    for (int i = 0; i < N; ++i)
      if (out[i].offsets && out[i].length >= 0) out[i].offsets[0] = 0;
    return FORY_OK;
  }
  for (int64_t k = 0; k < n; ++k)
    if (host_row_offsets[k + 1] < host_row_offsets[k]) return fail_host(FORY_ERR_CORRUPT, "row offsets decrease");
  if (host_row_offsets[0] < 0) return fail_host(FORY_ERR_CORRUPT, "row offsets decrease");
  for (int i = 0; i < N; ++i)
    if (has_offsets(c->kind[i]) && !out[i].offsets)
      return fail_host(FORY_ERR_INVALID_ARGUMENT, "output column " + std::to_string(i) + " needs offsets");
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  call_extent(c, host_rows + host_row_offsets[0], host_row_offsets[n] - host_row_offsets[0]);
  for (int i = 0; i < N; ++i) {  // caller-sized outputs
    const int64_t len = out[i].length;
    if (len <= 0) continue;
    if (c->kind[i] == kKindBytes) call_extent(c, out[i].values, out[i].capacity);
    else if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) call_extent(c, out[i].values, len * c->width[i]);
    if (has_offsets(c->kind[i])) call_extent(c, out[i].offsets, (len + 1) * 4);
    if (c->nullable[i]) call_extent(c, out[i].validity, (len + 7) / 8);
  }
  const int64_t chunks = (n + c->chunk - 1) / c->chunk;
  const int64_t ws_bytes = fory_rowfmt_workspace_bytes(c->plan, std::min(n, c->chunk));
  rc = hip_check(hipMemsetAsync(c->vstatus, 0, 8, c->s_k), "hipMemsetAsync");
  if (!rc) rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
  if (rc) return rc;
  std::vector<char> wv(N, 0);
  for (int i = 0; i < N; ++i) wv[i] = c->nullable[i] && out[i].validity;
  std::vector<int64_t> E(N, 0), VB(N, 0);  // elements / value bytes of the chunks before
  struct Stash { int col; int64_t byte; int64_t slot; };
  std::vector<Stash> stash;
  // context-owned pinned scratch (grown, not allocated per call):
  // [N int32 level totals][chunks x N validity stash bytes]
  rc = ensure_hpin(c, 4 * (int64_t)N + chunks * N + 16);
  if (rc) return rc;
  uint8_t* pin = c->hpin;
  int32_t* tpin = reinterpret_cast<int32_t*>(pin);
  uint8_t* spin = pin + 4 * N;
  bool overflow = false;
  int64_t crow[2] = {};
  int64_t* d_offs[2] = {};

  auto prefetch = [&](int64_t k) -> int {  // rows + relative offsets of chunk k (s_in)
    const int b = (int)(k & 1);
    fory_host_ctx::VarSlot& S = c->vs[b];
    const int64_t a = k * c->chunk, rows = std::min(c->chunk, n - a);
    const int64_t lo = host_row_offsets[a], hi = host_row_offsets[a + rows];
    const int64_t run = align_up(hi - lo + 16), need = run + align_up((rows + 1) * 8);
    int r = FORY_OK;
    if (S.used) r = hip_check(hipStreamWaitEvent(c->s_in, c->ev_k[b], 0), "hipStreamWaitEvent");  // k-2 decoded
    if (!r && S.used) r = hip_check(hipEventSynchronize(c->ev_in[b]), "hipEventSynchronize");  // its pin copy left
    if (!r && need > S.rows_bytes) {
      if (S.used) r = hip_check(hipEventSynchronize(c->ev_k[b]), "hipEventSynchronize");
      if (S.rows) (void)hipFree(S.rows);
      S.rows = nullptr, S.rows_bytes = 0;
      const int64_t sz = align_up(need + need / 4);
      if (!r) r = hip_check(hipMalloc(&S.rows, (size_t)sz), "hipMalloc(host ctx chunk rows)");
      if (!r) S.rows_bytes = sz;
    }
    if (!r && S.pin_words < rows + 1) {
      if (S.pin) (void)hipHostFree(S.pin);
      S.pin = nullptr, S.pin_words = 0;
      r = hip_check(hipHostMalloc(reinterpret_cast<void**>(&S.pin), (size_t)(c->chunk + 1) * 8, hipHostMallocCoherent),
                    "hipHostMalloc(row offsets)");
      if (!r) S.pin_words = c->chunk + 1;
    }
    if (r) return r;
    for (int64_t i = 0; i <= rows; ++i) S.pin[i] = host_row_offsets[a + i] - lo;
    d_offs[b] = reinterpret_cast<int64_t*>(S.rows + run);
    if (hi > lo) r = hcopy(c, S.rows, host_rows + lo, (size_t)(hi - lo), hipMemcpyHostToDevice, c->s_in, "H2D rows");
    if (!r) r = hcopy(c, d_offs[b], S.pin, (size_t)(rows + 1) * 8, hipMemcpyHostToDevice, c->s_in, "H2D row offsets");
    if (!r) r = hip_check(hipEventRecord(c->ev_in[b], c->s_in), "hipEventRecord");
    if (!r) r = verify_pieces(c, c->s_in, k);
    crow[b] = rows;
    return r;
  };

  rc = prefetch(0);
  for (int64_t k = 0; k < chunks && !rc; ++k) {
    const int b = (int)(k & 1);
    fory_host_ctx::VarSlot& S = c->vs[b];
    if (k + 1 < chunks) rc = prefetch(k + 1);
    const int64_t rows = crow[b];
    int32_t* status = c->vstatus + b;
    // sizes, level by level (decode_var_stage): counts of the columns known so far
    if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_in[b], 0), "hipStreamWaitEvent");
    if (!rc && S.used) rc = hip_check(hipStreamWaitEvent(c->s_k, c->ev_out[b], 0), "hipStreamWaitEvent");
    std::vector<int64_t> cnt(N, -1), vbytes(N, 0);
    auto resolve = [&]() {
      for (int i = 0; i < N; ++i) {
        const int p = c->parent[i];
        if (cnt[i] >= 0) continue;
        if (p < 0) cnt[i] = rows;
        else if (cnt[p] >= 0 && c->kind[p] == kKindStruct) cnt[i] = cnt[p];
      }
    };
    resolve();
    std::vector<fory_column> d;
    void* ws = nullptr;
    std::vector<char> nov(N, 0);
    std::vector<int64_t> vb0(N, 0), kc(N);
    for (int pass = 0; pass < 20 && !rc; ++pass) {
      for (int i = 0; i < N; ++i) kc[i] = cnt[i];
      const int64_t need = carve(c, nullptr, kc, vb0, nov, rows, nullptr, nullptr, nullptr, ws_bytes, nullptr);
      if (need > S.dev_bytes) {
        rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
        if (!rc && S.used) rc = hip_check(hipEventSynchronize(c->ev_out[b]), "hipEventSynchronize");
        if (S.dev) (void)hipFree(S.dev);
        S.dev = nullptr, S.dev_bytes = 0;
        const int64_t sz = align_up(need + need / 4);
        if (!rc) rc = hip_check(hipMalloc(&S.dev, (size_t)sz), "hipMalloc(host ctx chunk slot)");
        if (!rc) S.dev_bytes = sz;
        if (rc) break;
      }
      carve(c, S.dev, kc, vb0, nov, rows, &d, nullptr, &ws, ws_bytes, nullptr);
      for (int i = 0; i < N; ++i) {
        d[i].values = nullptr;
        d[i].capacity = 0;
        if (kc[i] < 0) d[i] = fory_column{};
      }
      rc = fory_rowfmt_decode_sizes(c->plan, S.rows, d_offs[b], rows, frame, d.data(), status, ws, ws_bytes, c->s_k);
      for (int i = 0; i < N && !rc; ++i)
        if (d[i].offsets && kc[i] >= 0)
          rc = hip_check(hipMemcpyAsync(tpin + i, d[i].offsets + kc[i], 4, hipMemcpyDeviceToHost, c->s_k), "D2H totals");
      if (!rc) rc = fory_rowfmt_read_status(status, c->s_k);  // synchronises s_k
      const int32_t* tot = tpin;
      if (rc) break;
      bool changed = false;
      for (int i = 0; i < N; ++i) {
        if (!has_offsets(c->kind[i]) || kc[i] < 0) continue;
        if (c->kind[i] == kKindBytes) vbytes[i] = tot[i];
        else
          for (int j = 0; j < N; ++j)
            if (c->parent[j] == i && cnt[j] < 0) cnt[j] = tot[i], changed = true;
      }
      resolve();
      if (!changed) break;
    }
    if (rc) break;
    for (int i = 0; i < N; ++i) {
      if (cnt[i] < 0) cnt[i] = 0, kc[i] = -1;  // (no buffers in the sizes layout)
      if (c->kind[i] == kKindFixed || c->kind[i] == kKindBool) vbytes[i] = cnt[i] * c->width[i];
      host_counts[i] += cnt[i];
      host_bytes[i] += vbytes[i];
      const int64_t vcap = c->kind[i] == kKindBytes ? out[i].capacity : (out[i].length) * c->width[i];
      if (E[i] + cnt[i] > out[i].length || (vbytes[i] > 0 && VB[i] + vbytes[i] > vcap) ||
          (vbytes[i] > 0 && !out[i].values))
        overflow = true;
    }
    if (!overflow) {
      // output region after the sizes layout: values, validity, shifted validity
      const int64_t at0 = carve(c, nullptr, kc, vb0, nov, rows, nullptr, nullptr, nullptr, ws_bytes, nullptr);
      int64_t at = at0;
      std::vector<int64_t> o_val(N, -1), o_vld(N, -1), o_sh(N, -1);
      for (int i = 0; i < N; ++i) {
        if (vbytes[i] > 0) o_val[i] = at, at += align_up(vbytes[i] + kSlack);
        if (wv[i]) {
          o_vld[i] = at, at += align_up(validity_bytes(cnt[i] > 0 ? cnt[i] : 1) + kSlack);
          if (E[i] & 7) o_sh[i] = at, at += align_up(cnt[i] / 8 + 2 + kSlack);
        }
      }
      if (at > S.dev_bytes) {  // grow, keeping the sizes layout's offsets
        uint8_t* nd = nullptr;
        const int64_t sz = align_up(at + at / 4);
        rc = hip_check(hipMalloc(&nd, (size_t)sz), "hipMalloc(host ctx chunk slot)");
        if (!rc) rc = hip_check(hipMemcpyAsync(nd, S.dev, (size_t)at0, hipMemcpyDeviceToDevice, c->s_k), "D2D");
        if (!rc) rc = hip_check(hipStreamSynchronize(c->s_k), "hipStreamSynchronize");
        if (rc) {
          if (nd) (void)hipFree(nd);
          break;
        }
        (void)hipFree(S.dev);
        S.dev = nd, S.dev_bytes = sz;
        carve(c, S.dev, kc, vb0, nov, rows, &d, nullptr, &ws, ws_bytes, nullptr);
      }
      for (int i = 0; i < N && !rc; ++i) {
        d[i].values = o_val[i] >= 0 ? S.dev + o_val[i] : nullptr;
        d[i].capacity = vbytes[i];
        d[i].length = cnt[i];
        d[i].validity = o_vld[i] >= 0 ? S.dev + o_vld[i] : nullptr;
        if (d[i].validity)
          rc = hip_check(hipMemsetAsync(d[i].validity, 0, (size_t)validity_bytes(cnt[i] > 0 ? cnt[i] : 1), c->s_k),
                         "hipMemsetAsync");
      }
      if (!rc)
        rc = fory_rowfmt_decode(c->plan, S.rows, d_offs[b], rows, frame, d.data(), status, ws, ws_bytes, c->s_k);
      for (int i = 0; i < N && !rc; ++i) {  // batch positions
        if (d[i].offsets) {
          int64_t base = 0, span = 0;  // batch position of the chunk's first element / value byte, chunk total
          if (c->kind[i] == kKindBytes) {
            base = VB[i], span = vbytes[i];
          } else {
            for (int j = 0; j < N; ++j)
              if (c->parent[j] == i) {
                base = E[j], span = cnt[j];
                break;
              }
          }
          if (base + span > INT32_MAX) {  // the moved offsets end at base + span
            rc = fail_host(FORY_ERR_CAPACITY, "column " + std::to_string(i) + " exceeds int32 offsets");
            break;
          }
          rc = hip_check(fory_amd::launch_offsets_add(d[i].offsets, cnt[i], (int32_t)base, c->s_k), "offsets_add");
        }
        if (!rc && o_sh[i] >= 0)
          rc = hip_check(fory_amd::launch_bits_shift(d[i].validity, cnt[i], S.dev + o_sh[i], (int)(E[i] & 7), c->s_k),
                         "bits_shift");
      }
      if (!rc) rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
      if (!rc) rc = hip_check(hipStreamWaitEvent(c->s_out, c->ev_k[b], 0), "hipStreamWaitEvent");
      for (int i = 0; i < N && !rc; ++i) {
        const fory_column& h = out[i];
        if (d[i].values && vbytes[i] > 0) {
          const int64_t dst = c->kind[i] == kKindBytes ? VB[i] : E[i] * c->width[i];
          rc = hcopy(c, static_cast<uint8_t*>(h.values) + dst, d[i].values, (size_t)vbytes[i], hipMemcpyDeviceToHost,
                     c->s_out, "D2H values");
        }
        if (!rc && d[i].offsets)
          rc = hcopy(c, h.offsets + E[i], d[i].offsets, (size_t)(cnt[i] + 1) * 4, hipMemcpyDeviceToHost, c->s_out,
                     "D2H offsets");
        if (!rc && d[i].validity && cnt[i] > 0) {
          const int sh = (int)(E[i] & 7);
          const int64_t nbytes = (sh + cnt[i] + 7) >> 3;
          const uint8_t* src = sh ? S.dev + o_sh[i] : d[i].validity;
          if (sh) {  // byte 0 is shared with the chunk before: OR-ed at the end
            const int64_t slot = k * N + i;
            stash.push_back(Stash{i, E[i] >> 3, slot});
            rc = hip_check(hipMemcpyAsync(spin + slot, src, 1, hipMemcpyDeviceToHost, c->s_out), "D2H validity");
          }
          if (!rc && nbytes > (sh ? 1 : 0))
            rc = hcopy(c, h.validity + (E[i] >> 3) + (sh ? 1 : 0), src + (sh ? 1 : 0), (size_t)(nbytes - (sh ? 1 : 0)),
                       hipMemcpyDeviceToHost, c->s_out, "D2H validity");
        }
      }
      if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_out), "hipEventRecord");
    } else {  // sized only
      rc = hip_check(hipEventRecord(c->ev_k[b], c->s_k), "hipEventRecord");
      if (!rc) rc = hip_check(hipEventRecord(c->ev_out[b], c->s_k), "hipEventRecord");
    }
    S.used = true;
    for (int i = 0; i < N; ++i) E[i] += cnt[i], VB[i] += vbytes[i];
  }
  const int rc_sync = sync_all(c);  // (drains the staged D2H pieces before the OR below)
  if (!rc && !rc_sync && !overflow)
    for (const Stash& st : stash) out[st.col].validity[st.byte] |= spin[st.slot];
  if (rc) return rc;
  if (rc_sync) return rc_sync;
  for (int b = 0; b < 2 && !rc; ++b) rc = fory_rowfmt_read_status(c->vstatus + b, c->s_k);
  if (rc) return rc;
  if (overflow) return fail_host(FORY_ERR_CAPACITY, "output columns too small (host_counts / host_bytes: the sizes)");
  return FORY_OK;
}

}  // namespace

extern "C" int fory_rowfmt_host_decode_var_into(fory_host_ctx* c, const void* host_rows, const int64_t* host_row_offsets,
                                                int64_t n, int32_t frame, const fory_column* host_out_cols,
                                                int64_t* host_counts, int64_t* host_bytes) {
  if (!c) return fail_host(FORY_ERR_INVALID_ARGUMENT, "ctx is null");
  if (!c->varlen) return fail_host(FORY_ERR_INVALID_ARGUMENT, "fixed-width plan: use fory_rowfmt_host_decode");
  if (n < 0) return fail_host(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (!host_row_offsets || !host_counts || !host_bytes || !host_out_cols || (n > 0 && !host_rows))
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "host rows, row offsets, output columns or size outputs null");
  return host_decode_var_into(c, static_cast<const uint8_t*>(host_rows), host_row_offsets, n, frame, host_out_cols,
                              host_counts, host_bytes);
}

// Library-internal, for tests (not in the public header): how hcopy would move
// [p, p + bytes) — 1 = one async DMA (pinned over the whole range), 0 = staged — and
// how many pieces a context has staged so far.
extern "C" int fory_rowfmt_internal_host_copy_path(const void* p, int64_t bytes) {
  return bytes > 0 && pinned_range(p, (size_t)bytes) ? 1 : 0;
}

extern "C" int64_t fory_rowfmt_internal_host_staged_pieces(const fory_host_ctx* c) { return c ? c->stage.pieces : -1; }
// Call-scoped registrations a context made over its life: out[0] count, out[1] bytes,
// out[2] microseconds spent registering; returns the number of call-scoped registrations
// alive in the process right now (0 between calls).
extern "C" int fory_rowfmt_internal_host_call_regs(const fory_host_ctx* c, int64_t* out) {
  if (c && out) {
    out[0] = c->reg_calls;
    out[1] = c->reg_bytes;
    out[2] = (int64_t)(c->reg_ms * 1000.0);
  }
  std::lock_guard<std::mutex> lock(g_reg_mu);
  return (int)g_tmp.size();
}
// Library-internal, for tests of the copy machinery alone: one call's worth of copies
// through hcopy, then the end-of-call drain. The caller buffers decl[0..ndecl) are declared
// for the call, as the host entry points declare theirs, so they are registered for it.
// Staged pieces go through the ring and small pieces through the small buffers.
// kinds[i]: 1 = H2D, 2 = D2H; streams[i]: 0 = in, 1 = kernels, 2 = out. On the GPU it is one
// more parity check. On the CPU, tests/c/host_copy_mock.cpp links host.cpp against a
// mock HIP runtime whose DMAs run late, so a staging block rewritten, or a registration
// dropped, before its DMA ran shows up as wrong bytes or a logged violation.
// flags & 1: return right after queuing the copies, as an error return does (CallScope then
// drains them).
extern "C" int fory_rowfmt_internal_host_copies(fory_host_ctx* c, int32_t n, void* const* dst,
                                                const void* const* src, const int64_t* bytes,
                                                const int32_t* kinds, const int32_t* streams, int32_t ndecl,
                                                const void* const* decl, const int64_t* decl_bytes, int32_t flags) {
  if (!c || n < 0 || (n > 0 && (!dst || !src || !bytes || !kinds || !streams)) || ndecl < 0 ||
      (ndecl > 0 && (!decl || !decl_bytes)))
    return fail_host(FORY_ERR_INVALID_ARGUMENT, "host_copies: bad arguments");
  int rc = hip_check(hipSetDevice(c->device), "hipSetDevice");
  if (rc) return rc;
  CallScope scope(c);
  for (int32_t i = 0; i < ndecl; ++i) call_extent(c, decl[i], decl_bytes[i]);
  for (int32_t i = 0; i < n && !rc; ++i) {
    if (kinds[i] != 1 && kinds[i] != 2) return fail_host(FORY_ERR_INVALID_ARGUMENT, "host_copies: kind");
    hipStream_t s = streams[i] == 0 ? c->s_in : (streams[i] == 1 ? c->s_k : c->s_out);
    rc = hcopy(c, dst[i], src[i], (size_t)bytes[i], kinds[i] == 1 ? hipMemcpyHostToDevice : hipMemcpyDeviceToHost, s,
               "host_copies");
  }
  if (flags & 1) return rc;
  const int rs = sync_all(c);
  return rc ? rc : rs;
}

// The staged copies' host memcpy (CopyPool), for a CPU test of its split.
extern "C" void fory_rowfmt_internal_pool_copy(void* dst, const void* src, int64_t n) {
  CopyPool::get().copy(dst, src, (size_t)n);
}

// Library-internal, for tests: round 2's classification (the first byte's attribute
// only), kept to show the straddling-range hazard it had next to pinned_range's answer.
extern "C" int fory_rowfmt_internal_host_first_byte_pinned(const void* p) {
  hipPointerAttribute_t a{};
  if (!p || hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return a.type != hipMemoryTypeUnregistered ? 1 : 0;
}
