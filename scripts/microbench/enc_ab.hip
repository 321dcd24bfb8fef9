// enc_ab.hip — the Struct104 encode's box-to-box spread: in one process,
// alternating, on 64Mi records, the product encode v5 (XCD-blocked tile order, non-temporal
// column loads and row stores) against the write-side variables the decode does not share:
// dispatch tile order, plain (temporal) row stores, both; decode v5 as the reference.
// Every variant's rows are compared with the product's. Build (from the repo root):
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -Ifury_amd/csrc scripts/microbench/enc_ab.hip \
//     fury_amd/csrc/launch_state.cpp -o scripts/microbench/bin/enc_ab
// Prints one JSON line per run: variant, round, ms per launch (mean of 10 after 3 warm-ups).
#include "../../fury_amd/csrc/fixed.hip"

#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e = (x);                                                        \
    if (e != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

using namespace fory_amd;

__global__ void fill_kernel(uint64_t* p, int64_t n, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    x ^= x >> 31;
    x *= 0xBF58476D1CE4E5B9ull;
    p[i] = x ^ (x >> 29);
  }
}

__global__ void diff_kernel(const uint64_t* a, const uint64_t* b, int64_t n, unsigned long long* bad) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    if (a[i] != b[i]) atomicAdd(bad, 1ull);
}

template <typename F>
static double time_ms(F launch, int reps = 10) {
  for (int i = 0; i < 3; ++i) launch();
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  CHECK(hipEventRecord(a, 0));
  for (int i = 0; i < reps; ++i) launch();
  CHECK(hipEventRecord(b, 0));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  CHECK(hipGetLastError());
  return ms / reps;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : (64ll << 20);
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  std::vector<std::string> names;
  for (int i = 0; i < 104; ++i) names.push_back("f" + std::to_string(i));
  std::sort(names.begin(), names.end());
  std::vector<int> width(104);
  for (int s = 0; s < 104; ++s) {
    const int idx = atoi(names[s].c_str() + 1);
    width[s] = (idx % 4 == 1 || idx % 4 == 3) ? 8 : 4;
  }
  std::vector<FixedFieldDev> tab;
  std::vector<uint8_t*> cols(104), dcols(104);
  for (int s = 0; s < 104; ++s) {
    CHECK(hipMalloc(&cols[s], n * width[s]));
    CHECK(hipMalloc(&dcols[s], n * width[s]));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t*)cols[s], n * width[s] / 8, (uint64_t)s);
    FixedFieldDev f{};
    f.values = cols[s];
    f.out_values = dcols[s];
    f.width = width[s];
    f.slot = s;
    tab.push_back(f);
  }
  std::stable_sort(tab.begin(), tab.end(), [](const FixedFieldDev& a, const FixedFieldDev& b) { return a.width > b.width; });
  FixedFieldDev* dtab;
  CHECK(hipMalloc(&dtab, tab.size() * sizeof(FixedFieldDev)));
  CHECK(hipMemcpy(dtab, tab.data(), tab.size() * sizeof(FixedFieldDev), hipMemcpyHostToDevice));
  FixedLaunch L{};
  L.fields = dtab;
  L.num_fields = 104;
  L.bitmap_bytes = 16;
  L.fixed_size = 848;
  L.stride = 848;
  L.schema_hash = 2926194988097786773ll;
  L.num_rows = n;
  L.group[0] = 0;
  L.group[1] = 52;
  L.group[2] = L.group[3] = L.group[4] = 104;
  L.rot4 = v5_rotation(848, 0, 16, 4, false);
  L.rot8 = v5_rotation(848, 0, 16, 8, false);
  L.drot4 = L.drot8 = 31;
  L.cols_aligned16 = 1;
  const int64_t row_bytes = n * 848;
  uint8_t *rows, *rows2;
  CHECK(hipMalloc(&rows, row_bytes));
  CHECK(hipMalloc(&rows2, row_bytes));
  int32_t* status;
  CHECK(hipMalloc(&status, 4));
  CHECK(hipMemset(status, 0, 4));
  unsigned long long* dbad;
  CHECK(hipMalloc(&dbad, 8));
  CHECK(hipDeviceSynchronize());
  const int64_t full = n / 64;
  auto enc = [&](auto* k, uint8_t* out, bool xcd) {
    raise_lds_cap(k);
    const size_t lds = (size_t)64 * 848;
    const int64_t g = persistent_grid(k, lds, full, 1024);
    const int64_t c = xcd ? full / 8 : 0;
    return [=]() { hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(1024), lds, 0, L, L.fields, out, full, c); };
  };
  auto* kp = &encode_fixed_v5_kernel<64, 1024, 3, 0, 1, false>;  // round 5's product: nt loads, nt stores
  auto* kw = &encode_fixed_v5_kernel<64, 1024, 3, 0, 5, false>;  // plain row stores
  auto* kq = &encode_fixed_v5_kernel<64, 1024, 3, 0, 4, false>;  // plain loads, plain stores
  auto product = enc(kp, rows, true);
  product();
  CHECK(hipDeviceSynchronize());
  struct V {
    const char* name;
    std::function<void()> f;
  };
  std::vector<V> vs = {{"r5: xcd-blocked, nt loads, nt stores", product},
                       {"dispatch order, nt stores", enc(kp, rows2, false)},
                       {"xcd-blocked, nt loads, plain stores", enc(kw, rows2, true)},
                       {"xcd-blocked, plain loads, plain stores", enc(kq, rows2, true)},
                       {"dispatch order, plain stores", enc(kw, rows2, false)}};
  auto dec = [&](auto* kd) {
    raise_lds_cap(kd);
    const int64_t gd = persistent_grid(kd, (size_t)64 * 848, full, 1024);
    return [=]() { hipLaunchKernelGGL(kd, dim3((unsigned)gd), dim3(1024), (size_t)64 * 848, 0, L, L.fields, rows, full, status); };
  };
  std::vector<V> ds = {{"decode: nt loads, nt stores (r5)", dec(&decode_fixed_v5_kernel<64, 1024, 4, 3, 0, 0, false>)},
                       {"decode: nt loads, plain stores", dec(&decode_fixed_v5_kernel<64, 1024, 4, 3, 0, 4, false>)},
                       {"decode: plain loads, plain stores", dec(&decode_fixed_v5_kernel<64, 1024, 4, 3, 0, 12, false>)},
                       {"decode: plain loads, nt stores", dec(&decode_fixed_v5_kernel<64, 1024, 4, 3, 0, 8, false>)}};
  char bus[64] = {0};
  (void)hipDeviceGetPCIBusId(bus, sizeof bus, 0);
  for (int r = 0; r < rounds; ++r) {
    for (auto& v : vs) {
      const double ms = time_ms(v.f);
      unsigned long long bad = 0;
      if (v.name != vs[0].name) {
        CHECK(hipMemset(dbad, 0, 8));
        hipLaunchKernelGGL(diff_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t*)rows, (const uint64_t*)rows2,
                           row_bytes / 8, dbad);
        CHECK(hipMemcpy(&bad, dbad, 8, hipMemcpyDeviceToHost));
      }
      printf("{\"bus\": \"%s\", \"round\": %d, \"variant\": \"%s\", \"ms\": %.4f, \"frac8000\": %.4f, \"mismatch_words\": %llu}\n",
             bus, r, v.name, ms, 98784247808.0 / (ms * 1e-3) / 8e12, bad);
      fflush(stdout);
    }
    for (auto& v : ds) {  // (every variant decodes the same rows into the same columns)
      const double ms = time_ms(v.f);
      printf("{\"bus\": \"%s\", \"round\": %d, \"variant\": \"%s\", \"ms\": %.4f, \"frac8000\": %.4f}\n", bus, r,
             v.name, ms, 98784247808.0 / (ms * 1e-3) / 8e12);
      fflush(stdout);
    }
  }
  return 0;
}
