// host_copy_mock — the host path's copy machinery (fury_amd/csrc/host.cpp: the staging ring,
// the small-piece buffers, call-scoped registration of caller buffers, the end-of-call drain)
// on the CPU, against a mock HIP runtime whose DMAs run LATE.
//
// An async copy is queued on its stream and runs only when something waits for it
// (hipEventSynchronize, hipStreamSynchronize, hipStreamWaitEvent) or when the seeded random
// progress model picks it. Its host bytes are read or written when it runs, not when it is
// queued. So:
//   - a staging block rewritten before the H2D that reads it has run gives wrong device bytes;
//   - an owed D2H host copy made before its DMA has run gives wrong host bytes.
// The mock also logs a violation for each of these:
//   - a DMA queued on pageable host memory;
//   - a DMA that spans two pinned ranges, or runs outside a device allocation;
//   - a DMA that runs after its host range was unregistered or freed;
//   - an unregister or free while a queued DMA still references the range.
// Test infrastructure only ("a CPU test of the staging ring's block-reuse
// order"); built by `make tests/c/host_copy_mock`, run by tests/test_host_copy_mock.py.
// host.cpp is compiled with small staging and registration sizes here (Makefile), so a few
// MiB exercise block reuse, small-buffer switching and registration pieces.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <string>
#include <vector>

#include "../../include/fory_rowfmt.h"

// ---------------------------------------------------------------- mock runtime
namespace {

struct Op {
  uint8_t* dst;
  const uint8_t* src;
  size_t n;
  int memset_value;  // >= 0: a memset of dst
  const uint8_t* host;  // the host side of a copy (nullptr: device-only op)
};

struct Range {
  size_t n;
  int kind;  // 1 hipHostMalloc, 2 hipHostRegister, 3 hipMalloc
};

std::mutex g_mu;  // (the library's CopyPool threads never call the runtime; one lock is plenty)
std::map<uintptr_t, Range> g_ranges;
std::vector<std::string> g_violations;
std::mt19937_64 g_rng(1);
int g_progress = 4;  // per queued op: run up to this many ops of random streams (0: only on waits)
uint64_t g_ops = 0;

void violation(const std::string& s) {
  if (g_violations.size() < 50) g_violations.push_back(s);
  else if (g_violations.size() == 50) g_violations.push_back("...");
}

const Range* find(uintptr_t a, uintptr_t* base) {
  auto it = g_ranges.upper_bound(a);
  if (it == g_ranges.begin()) return nullptr;
  --it;
  if (a >= it->first && a < it->first + it->second.n) {
    *base = it->first;
    return &it->second;
  }
  return nullptr;
}

// [p, p + n) inside one range of one of the kinds in mask (bit k: kind k)?
bool inside(const void* p, size_t n, int mask) {
  uintptr_t b = 0;
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const Range* r = find(a, &b);
  return r && ((mask >> r->kind) & 1) && a + n <= b + r->n;
}

}  // namespace

struct ihipStream_t {
  std::deque<Op> q;
  uint64_t issued = 0, done = 0;
};
struct ihipEvent_t {
  ihipStream_t* s = nullptr;
  uint64_t seq = 0;
};

namespace {

std::vector<ihipStream_t*> g_streams;

void run_one(ihipStream_t* s) {
  Op op = s->q.front();
  s->q.pop_front();
  ++s->done;
  if (op.host && !inside(op.host, op.n, (1 << 1) | (1 << 2)))
    violation("a DMA ran after its host range was unregistered or freed");
  if (op.memset_value >= 0) std::memset(op.dst, op.memset_value, op.n);
  else std::memmove(op.dst, op.src, op.n);
}

void run_until(ihipStream_t* s, uint64_t seq) {
  while (s && s->done < seq && !s->q.empty()) run_one(s);
}

void progress() {
  if (g_streams.empty()) return;
  const int k = (int)(g_rng() % (uint64_t)(g_progress + 1));
  for (int i = 0; i < k; ++i) {
    ihipStream_t* s = g_streams[g_rng() % g_streams.size()];
    if (!s->q.empty()) run_one(s);
  }
}

bool referenced(uintptr_t a, size_t n) {
  for (ihipStream_t* s : g_streams)
    for (const Op& op : s->q) {
      const uintptr_t lo[2] = {reinterpret_cast<uintptr_t>(op.dst), reinterpret_cast<uintptr_t>(op.src)};
      for (uintptr_t x : lo)
        if (x && x < a + n && a < x + op.n) return true;
    }
  return false;
}

}  // namespace

extern "C" {

hipError_t hipSetDevice(int) { return hipSuccess; }
hipError_t hipGetLastError(void) { return hipSuccess; }
const char* hipGetErrorString(hipError_t e) { return e == hipSuccess ? "no error" : "mock error"; }

hipError_t hipStreamCreateWithFlags(hipStream_t* s, unsigned int) {
  std::lock_guard<std::mutex> l(g_mu);
  *s = new ihipStream_t();
  g_streams.push_back(*s);
  return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t s) {
  std::lock_guard<std::mutex> l(g_mu);
  run_until(s, UINT64_MAX);
  g_streams.erase(std::remove(g_streams.begin(), g_streams.end(), s), g_streams.end());
  delete s;
  return hipSuccess;
}
hipError_t hipStreamSynchronize(hipStream_t s) {
  std::lock_guard<std::mutex> l(g_mu);
  run_until(s, UINT64_MAX);
  return hipSuccess;
}
hipError_t hipStreamWaitEvent(hipStream_t, hipEvent_t e, unsigned int) {
  std::lock_guard<std::mutex> l(g_mu);
  if (e) run_until(e->s, e->seq);  // (conservative: the producer's work runs now)
  return hipSuccess;
}
hipError_t hipEventCreateWithFlags(hipEvent_t* e, unsigned) {
  *e = new ihipEvent_t();
  return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t e) {
  delete e;
  return hipSuccess;
}
hipError_t hipEventRecord(hipEvent_t e, hipStream_t s) {
  std::lock_guard<std::mutex> l(g_mu);
  e->s = s;
  e->seq = s ? s->issued : 0;
  return hipSuccess;
}
hipError_t hipEventSynchronize(hipEvent_t e) {
  std::lock_guard<std::mutex> l(g_mu);
  run_until(e->s, e->seq);
  return hipSuccess;
}

hipError_t hipMalloc(void** p, size_t n) {
  std::lock_guard<std::mutex> l(g_mu);
  *p = std::aligned_alloc(256, (n + 255) / 256 * 256 + 256);
  g_ranges[reinterpret_cast<uintptr_t>(*p)] = Range{n, 3};
  return hipSuccess;
}
hipError_t hipFree(void* p) {
  if (!p) return hipSuccess;
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_ranges.find(reinterpret_cast<uintptr_t>(p));
  if (it == g_ranges.end()) return hipErrorInvalidValue;
  if (referenced(it->first, it->second.n)) violation("hipFree of device memory a queued DMA references");
  g_ranges.erase(it);
  std::free(p);
  return hipSuccess;
}
hipError_t hipHostMalloc(void** p, size_t n, unsigned int) {
  std::lock_guard<std::mutex> l(g_mu);
  *p = std::aligned_alloc(4096, (n + 4095) / 4096 * 4096);
  g_ranges[reinterpret_cast<uintptr_t>(*p)] = Range{n, 1};
  return hipSuccess;
}
hipError_t hipHostFree(void* p) {
  if (!p) return hipSuccess;
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_ranges.find(reinterpret_cast<uintptr_t>(p));
  if (it == g_ranges.end() || it->second.kind != 1) return hipErrorInvalidValue;
  if (referenced(it->first, it->second.n)) violation("hipHostFree of pinned memory a queued DMA references");
  g_ranges.erase(it);
  std::free(p);
  return hipSuccess;
}
hipError_t hipHostRegister(void* p, size_t n, unsigned int) {
  std::lock_guard<std::mutex> l(g_mu);
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  auto it = g_ranges.lower_bound(a);
  if (it != g_ranges.begin()) {
    auto pr = std::prev(it);
    if (pr->first + pr->second.n > a) return hipErrorHostMemoryAlreadyRegistered;
  }
  if (it != g_ranges.end() && it->first < a + n) return hipErrorHostMemoryAlreadyRegistered;
  g_ranges[a] = Range{n, 2};
  return hipSuccess;
}
hipError_t hipHostUnregister(void* p) {
  std::lock_guard<std::mutex> l(g_mu);
  auto it = g_ranges.find(reinterpret_cast<uintptr_t>(p));
  if (it == g_ranges.end() || it->second.kind != 2) return hipErrorHostMemoryNotRegistered;
  if (referenced(it->first, it->second.n)) violation("hipHostUnregister of a range a queued DMA references");
  g_ranges.erase(it);
  return hipSuccess;
}
hipError_t hipPointerGetAttributes(hipPointerAttribute_t* a, const void* p) {
  std::lock_guard<std::mutex> l(g_mu);
  std::memset(a, 0, sizeof(*a));
  uintptr_t b = 0;
  const Range* r = find(reinterpret_cast<uintptr_t>(p), &b);
  if (!r) {
    a->type = hipMemoryTypeUnregistered;
    return hipErrorInvalidValue;
  }
  a->type = r->kind == 3 ? hipMemoryTypeDevice : hipMemoryTypeHost;
  a->devicePointer = const_cast<void*>(p);  // (identity mapping)
  a->hostPointer = r->kind == 3 ? nullptr : const_cast<void*>(p);
  return hipSuccess;
}
hipError_t hipPointerGetAttribute(void* data, hipPointer_attribute attr, hipDeviceptr_t p) {
  std::lock_guard<std::mutex> l(g_mu);
  uintptr_t b = 0;
  const Range* r = find(reinterpret_cast<uintptr_t>(p), &b);
  if (!r) return hipErrorInvalidValue;
  if (attr == HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR) *static_cast<void**>(data) = reinterpret_cast<void*>(b);
  else if (attr == HIP_POINTER_ATTRIBUTE_RANGE_SIZE) *static_cast<size_t*>(data) = r->n;
  else return hipErrorInvalidValue;
  return hipSuccess;
}
hipError_t hipMemcpyAsync(void* dst, const void* src, size_t n, hipMemcpyKind kind, hipStream_t s) {
  std::lock_guard<std::mutex> l(g_mu);
  if (n == 0) return hipSuccess;
  const bool h2d = kind == hipMemcpyHostToDevice, d2h = kind == hipMemcpyDeviceToHost;
  const void* host = h2d ? src : (d2h ? dst : nullptr);
  const void* dev = h2d ? dst : (d2h ? src : dst);
  if (host && !inside(host, n, (1 << 1) | (1 << 2))) {
    violation("a DMA queued on host memory that is not pinned as one range");
    return hipErrorInvalidValue;
  }
  if (!inside(dev, n, 1 << 3)) {
    violation("a DMA outside a device allocation");
    return hipErrorInvalidValue;
  }
  s->q.push_back(Op{static_cast<uint8_t*>(dst), static_cast<const uint8_t*>(src), n, -1,
                    static_cast<const uint8_t*>(host)});
  ++s->issued;
  ++g_ops;
  progress();
  return hipSuccess;
}
hipError_t hipMemsetAsync(void* dst, int v, size_t n, hipStream_t s) {
  std::lock_guard<std::mutex> l(g_mu);
  s->q.push_back(Op{static_cast<uint8_t*>(dst), nullptr, n, v & 0xff, nullptr});
  ++s->issued;
  return hipSuccess;
}
hipError_t hipMemset(void* dst, int v, size_t n) {
  std::memset(dst, v, n);
  return hipSuccess;
}

// ---------------------------------------------------------------- the rest of the library
// host.cpp's calls into capi.cpp and the kernels: a varlen plan of one column; nothing here
// launches work (the copies-only entry point never reaches these).
static std::string g_err;
int fory_rowfmt_internal_set_error(int code, const char* msg) {
  g_err = msg ? msg : "";
  return code;
}
void fory_rowfmt_internal_retire_stream(void*) {}
int fory_rowfmt_plan_info(const fory_plan*, fory_plan_info* out) {
  std::memset(out, 0, sizeof(*out));
  out->num_fields = out->num_columns = 1;
  out->fixed_width = 0;
  out->row_size = -1;
  return FORY_OK;
}
int fory_rowfmt_internal_column_layout(const fory_plan*, int32_t* w, int32_t* nl) {
  w[0] = 8;
  nl[0] = 0;
  return FORY_OK;
}
int fory_rowfmt_internal_node_layout(const fory_plan*, int32_t* kind, int32_t* width, int32_t* nl, int32_t* parent) {
  kind[0] = 0, width[0] = 8, nl[0] = 0, parent[0] = -1;
  return FORY_OK;
}
int64_t fory_rowfmt_workspace_bytes(const fory_plan*, int64_t) { return 256; }
int64_t fory_rowfmt_index_workspace_bytes(const fory_plan*, int64_t, int64_t) { return 256; }
int fory_rowfmt_encoded_size(const fory_plan*, const fory_column*, int64_t, int32_t, int64_t*, void*, int64_t,
                             void*) {
  return FORY_ERR_UNSUPPORTED;
}
int fory_rowfmt_encode(const fory_plan*, const fory_column*, int64_t, int32_t, const int64_t*, void*, int64_t,
                       int32_t*, void*, int64_t, void*) {
  return FORY_ERR_UNSUPPORTED;
}
int fory_rowfmt_decode_sizes(const fory_plan*, const void*, const int64_t*, int64_t, int32_t, const fory_column*,
                             int32_t*, void*, int64_t, void*) {
  return FORY_ERR_UNSUPPORTED;
}
int fory_rowfmt_decode(const fory_plan*, const void*, const int64_t*, int64_t, int32_t, const fory_column*, int32_t*,
                       void*, int64_t, void*) {
  return FORY_ERR_UNSUPPORTED;
}
int fory_rowfmt_index_frames(const fory_plan*, const void*, int64_t, int64_t, int32_t, int64_t*, int32_t*, void*,
                             int64_t, void*) {
  return FORY_ERR_UNSUPPORTED;
}
int fory_rowfmt_read_status(const int32_t*, void*) { return FORY_OK; }

int fory_rowfmt_internal_host_copies(fory_host_ctx* c, int32_t n, void* const* dst, const void* const* src,
                                     const int64_t* bytes, const int32_t* kinds, const int32_t* streams, int32_t ndecl,
                                     const void* const* decl, const int64_t* decl_bytes, int32_t flags);
int fory_rowfmt_internal_host_call_regs(const fory_host_ctx* c, int64_t* out);
int64_t fory_rowfmt_internal_host_staged_pieces(const fory_host_ctx* c);
}  // extern "C"

namespace fory_amd {
bool host_verify_from_env() { return std::getenv("FORY_ROWFMT_HOST_VERIFY") != nullptr; }
hipError_t launch_offsets_add(int32_t*, int64_t, int32_t, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_bits_shift(const uint8_t*, int64_t, uint8_t*, int, hipStream_t) { return hipErrorNotSupported; }
}  // namespace fory_amd

// ---------------------------------------------------------------- scenarios
namespace {

struct Piece {
  void* dst;
  const void* src;
  int64_t n;
  int32_t kind, stream;
};

uint8_t* dev_alloc(size_t n) {
  void* p = nullptr;
  (void)hipMalloc(&p, n);
  return static_cast<uint8_t*>(p);
}

void fill(uint8_t* p, size_t n, uint64_t seed) {
  std::mt19937_64 r(seed);
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {
    const uint64_t x = r();
    std::memcpy(p + i, &x, 8);
  }
  for (; i < n; ++i) p[i] = (uint8_t)r();
}

int failures = 0;

void expect(bool ok, const char* scenario, const std::string& what) {
  if (!ok) {
    ++failures;
    std::printf("{\"scenario\": \"%s\", \"failed\": \"%s\"}\n", scenario, what.c_str());
  }
}

int run_call(fory_host_ctx* c, const std::vector<Piece>& ps, const std::vector<std::pair<const void*, int64_t>>& decl,
             int32_t flags) {
  std::vector<void*> d;
  std::vector<const void*> s, dp;
  std::vector<int64_t> b, db;
  std::vector<int32_t> k, st;
  for (const Piece& p : ps) d.push_back(p.dst), s.push_back(p.src), b.push_back(p.n), k.push_back(p.kind),
                                 st.push_back(p.stream);
  for (auto& x : decl) dp.push_back(x.first), db.push_back(x.second);
  return fory_rowfmt_internal_host_copies(c, (int32_t)ps.size(), d.data(), s.data(), b.data(), k.data(), st.data(),
                                          (int32_t)dp.size(), dp.data(), db.data(), flags);
}

// Random pieces between pageable host buffers and device buffers, both directions, sizes
// from a byte to several staging blocks, on random streams; per call, every host piece is
// distinct memory. After the call: every H2D's device bytes equal the source, every D2H's
// host bytes equal the device source.
// flags & 2 (test side, not passed on): the caller registers its first buffer itself
// (fory_rowfmt_host_register) before the call and unregisters it after; the call's own
// registration must decline it and its copies go direct through the caller's mapping.
void scenario_mixed(fory_host_ctx* c, const char* name, int calls, int pieces, size_t max_piece, uint64_t seed,
                    bool declare, int32_t flags) {
  std::mt19937_64 r(seed);
  for (int call = 0; call < calls; ++call) {
    std::vector<Piece> ps;
    std::vector<std::vector<uint8_t>> host;
    std::vector<uint8_t*> dev;
    std::vector<std::pair<const void*, int64_t>> decl;
    std::vector<size_t> off;  // a piece's offset into its (possibly shared) buffers
    // pieces share a few large host buffers (declared for the call when `declare`), at
    // random offsets: copies inside, across and at the edges of their page interiors
    const int nbuf = 3;
    std::vector<std::vector<uint8_t>> big(nbuf);
    std::vector<uint8_t*> bigdev(nbuf);
    std::vector<size_t> cursor(nbuf, 0);
    for (int i = 0; i < nbuf; ++i) {
      big[i].resize((size_t)pieces * max_piece / nbuf + 4096 + (size_t)(r() % 4096));
      bigdev[i] = dev_alloc(big[i].size());
      if (declare) decl.push_back({big[i].data(), (int64_t)big[i].size()});
      if ((flags & 2) && i == 0)
        expect(fory_rowfmt_host_register(big[0].data(), (int64_t)big[0].size()) == FORY_OK, name,
               "host_register: " + g_err);
    }
    std::vector<int> which;
    for (int i = 0; i < pieces; ++i) {
      const int w = (int)(r() % nbuf);
      size_t n = (size_t)(r() % 4 == 0 ? 1 + r() % 64 : 1 + r() % max_piece);
      if (cursor[w] + n > big[w].size()) n = big[w].size() - cursor[w];
      if (n == 0) continue;
      const int32_t kind = (int32_t)(1 + r() % 2), stream = (int32_t)(r() % 3);
      uint8_t* h = big[w].data() + cursor[w];
      uint8_t* d = bigdev[w] + cursor[w];
      if (kind == 1) fill(h, n, r());
      else fill(d, n, r());
      ps.push_back(kind == 1 ? Piece{d, h, (int64_t)n, kind, stream} : Piece{h, d, (int64_t)n, kind, stream});
      which.push_back(w);
      off.push_back(cursor[w]);
      cursor[w] += n + (size_t)(r() % 3 == 0 ? r() % 512 : 0);  // gaps now and then
    }
    // snapshot what each piece must end up as (H2D: the host source now; D2H: the device
    // source now), then make the call
    std::vector<std::vector<uint8_t>> want(ps.size());
    for (size_t i = 0; i < ps.size(); ++i) {
      const uint8_t* from = static_cast<const uint8_t*>(ps[i].src);
      want[i].assign(from, from + ps[i].n);
    }
    const int rc = run_call(c, ps, decl, flags & 1);
    expect(rc == FORY_OK, name, "call failed: " + g_err);
    for (size_t i = 0; i < ps.size(); ++i) {
      const uint8_t* got = static_cast<const uint8_t*>(ps[i].dst);
      if (std::memcmp(got, want[i].data(), (size_t)ps[i].n)) {
        size_t first = 0;
        while (got[first] == want[i][first]) ++first;
        expect(false, name,
               "call " + std::to_string(call) + " piece " + std::to_string(i) + " (" +
                   (ps[i].kind == 1 ? "H2D" : "D2H") + ", " + std::to_string(ps[i].n) + " bytes, stream " +
                   std::to_string(ps[i].stream) + "): first wrong byte " + std::to_string(first));
      }
    }
    int64_t regs[3];
    const int alive = fory_rowfmt_internal_host_call_regs(c, regs);
    expect(alive == 0, name, "call-scoped registrations alive after the call: " + std::to_string(alive));
    if (flags & 2)
      expect(fory_rowfmt_host_unregister(big[0].data()) == FORY_OK, name, "host_unregister: " + g_err);
    for (uint8_t* d : bigdev) (void)hipFree(d);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const uint64_t seed = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1;
  g_rng.seed(seed);
  fory_host_ctx* c = nullptr;
  int dummy_plan = 0;
  if (fory_rowfmt_host_ctx_create(reinterpret_cast<const fory_plan*>(&dummy_plan), 0, 1024, &c) != FORY_OK) {
    std::printf("{\"error\": \"ctx_create: %s\"}\n", g_err.c_str());
    return 2;
  }
  const struct {
    const char* name;
    int progress, calls, pieces;
    size_t max_piece;
    bool declare;
    int32_t flags;  // 1: the call returns before its drain, as an error return does
  } cases[] = {
      {"staged, DMAs only on waits", 0, 5, 60, 2u << 20, false, 0},
      {"staged, DMAs progress randomly", 4, 5, 60, 2u << 20, false, 0},
      {"small pieces across buffer switches, DMAs only on waits", 0, 3, 30000, 2048, false, 0},
      {"small pieces across buffer switches", 2, 3, 30000, 2048, false, 0},
      {"declared buffers, DMAs only on waits", 0, 5, 60, 2u << 20, true, 0},
      {"declared buffers, DMAs progress randomly", 4, 5, 60, 2u << 20, true, 0},
      {"declared buffers, small pieces", 2, 3, 6000, 8192, true, 0},
      {"declared buffers, the call returns before its drain", 0, 5, 60, 2u << 20, true, 1},
      {"declared buffers, one registered by the caller", 2, 4, 60, 2u << 20, true, 2},
  };
  for (const auto& k : cases) {
    g_progress = k.progress;
    const int before = failures;
    const size_t v0 = g_violations.size();
    scenario_mixed(c, k.name, k.calls, k.pieces, k.max_piece, seed * 7919 + (uint64_t)k.pieces, k.declare, k.flags);
    for (size_t i = v0; i < g_violations.size(); ++i) expect(false, k.name, "violation: " + g_violations[i]);
    std::printf("{\"scenario\": \"%s\", \"ok\": %s}\n", k.name, failures == before ? "true" : "false");
  }
  int64_t regs[3] = {0, 0, 0};
  fory_rowfmt_internal_host_call_regs(c, regs);
  const int64_t staged = fory_rowfmt_internal_host_staged_pieces(c);
  fory_rowfmt_host_ctx_destroy(c);
  std::printf("{\"summary\": true, \"seed\": %llu, \"failures\": %d, \"violations\": %zu, \"dma_ops\": %llu, "
              "\"staged_pieces\": %lld, \"call_registrations\": %lld, \"registered_bytes\": %lld}\n",
              (unsigned long long)seed, failures, g_violations.size(), (unsigned long long)g_ops, (long long)staged,
              (long long)regs[0], (long long)regs[1]);
  return failures || !g_violations.empty() ? 1 : 0;
}
