// fixed_ab.hip — in-process A/B of the fixed-width kernels on 64Mi Struct104 rows
// (diagnostic tool, not product code). It compiles the product kernels
// (fury_amd/csrc/fixed.hip) and instantiates variants of them: tile order
// (dispatch vs XCD-grouped, map_tile), tile / workgroup shapes. Every variant's output is
// compared with the baseline's before it is timed. Build:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../fury_amd/csrc fixed_ab.hip \
//     ../../fury_amd/csrc/launch_state.cpp -o fixed_ab
// Prints one JSON line per variant: ms per launch (mean of 10 after 3 warmups) and
// algorithmic GB/s (columns + rows bytes / time).
#include "../../fury_amd/csrc/fixed.hip"

#include <algorithm>
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

static unsigned long long diff(const void* a, const void* b, int64_t bytes) {
  unsigned long long* d;
  CHECK(hipMalloc(&d, 8));
  CHECK(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(diff_kernel, dim3(4096), dim3(256), 0, 0, (const uint64_t*)a, (const uint64_t*)b, bytes / 8, d);
  unsigned long long h = 0;
  CHECK(hipMemcpy(&h, d, 8, hipMemcpyDeviceToHost));
  CHECK(hipFree(d));
  return h;
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
  // Struct104 in schema order: names f0..f103 sorted as Java strings; f{4k} int,
  // f{4k+1} long, f{4k+2} float, f{4k+3} double (Struct.java:158-174)
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
  int64_t col_bytes = 0;
  for (int s = 0; s < 104; ++s) {
    CHECK(hipMalloc(&cols[s], n * width[s]));
    CHECK(hipMalloc(&dcols[s], n * width[s]));
    hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, (uint64_t*)cols[s], n * width[s] / 8, (uint64_t)s);
    col_bytes += n * width[s];
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
  const int64_t row_bytes = n * 848;
  uint8_t *rows, *rows2;
  CHECK(hipMalloc(&rows, row_bytes));
  CHECK(hipMalloc(&rows2, row_bytes));
  int32_t* status;
  CHECK(hipMalloc(&status, 4));
  CHECK(hipMemset(status, 0, 4));
  CHECK(hipDeviceSynchronize());
  const double algo = (double)(col_bytes + row_bytes);
  auto report = [&](const char* name, double ms, unsigned long long bad) {
    printf("{\"variant\": \"%s\", \"rows\": %lld, \"ms\": %.4f, \"GBps\": %.1f, \"frac8000\": %.4f, \"mismatch_words\": %llu}\n",
           name, (long long)n, ms, algo / (ms * 1e-3) / 1e9, algo / (ms * 1e-3) / 1e9 / 8000.0, bad);
    fflush(stdout);
  };
  const int64_t tiles = n / 64;
  // ---- encode (xcd: tiles per XCD run of the tile order, 0 = dispatch order)
  auto enc = [&](auto* k, int R, int WG, uint8_t* out, int64_t xcd) {
    raise_lds_cap(k);
    const size_t lds = (size_t)R * 848;
    const int64_t full = n / R;
    const int64_t g = persistent_grid(k, lds, full, WG);
    const int64_t c = xcd < 0 ? (g % 8 == 0 ? g / 8 : 0) : xcd;
    return [=]() { hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(WG), lds, 0, L, L.fields, out, full, c); };
  };
  auto base_enc = enc(&encode_fixed_v5_kernel<64, 512, 6, 0>, 64, 512, rows, 0);
  report("enc_r64_wg512 dispatch order", time_ms(base_enc), 0);
  auto run = [&](const char* name, auto* k, int R, int WG, int64_t xcd) {
    CHECK(hipMemset(rows2, 0, row_bytes));
    auto f = enc(k, R, WG, rows2, xcd);
    f();
    CHECK(hipDeviceSynchronize());
    const unsigned long long bad = diff(rows, rows2, row_bytes);
    report(name, time_ms(f), bad);
  };
  const int64_t T8 = n / 64 / 8;  // XCD-blocked: each XCD one contiguous eighth of the tiles
  run("enc_r64_wg1024_k3_xcd (product)", &encode_fixed_v5_kernel<64, 1024, 3, 0>, 64, 1024, -1);
  run("enc_r64_wg1024_k3_xcdblk", &encode_fixed_v5_kernel<64, 1024, 3, 0>, 64, 1024, T8);
  run("enc_r64_wg1024_k3_xcdblk_ntload", &encode_fixed_v5_kernel<64, 1024, 3, 0, 1>, 64, 1024, T8);
  run("enc_r64_wg1024_k3_xcd_ntload", &encode_fixed_v5_kernel<64, 1024, 3, 0, 1>, 64, 1024, -1);
  run("enc_r64_wg1024_k3_blocked_ntload", &encode_fixed_v5_kernel<64, 1024, 3, 0, 3>, 64, 1024, 0);
  run("enc_r128_wg1024_k6_blocked_ntload", &encode_fixed_v5_kernel<128, 1024, 6, 0, 3>, 128, 1024, 0);
  run("enc_r128_wg1024_k6_xcdblk", &encode_fixed_v5_kernel<128, 1024, 6, 0>, 128, 1024, n / 128 / 8);
  // ---- decode (inputs: the baseline's rows)
  auto dec = [&](int64_t xcd) {
    auto* k = &decode_fixed_kernel<64, 0, 12>;
    raise_lds_cap(k);
    FixedLaunch D = L;
    D.xcd_run = xcd;
    return [=]() { hipLaunchKernelGGL(k, dim3((unsigned)tiles), dim3(kWG), (size_t)64 * 848, 0, D, D.fields, rows, status); };
  };
  auto base_dec = dec(0);
  report("dec_tile64 dispatch order", time_ms(base_dec), diff(cols[0], dcols[0], n * width[0]));
  for (int m : {16, 64, 256}) {
    CHECK(hipMemset(dcols[5], 0, n * width[5]));
    auto f = dec(m);
    f();
    CHECK(hipDeviceSynchronize());
    const unsigned long long bad = diff(cols[5], dcols[5], n * width[5]);
    char name[64];
    snprintf(name, sizeof name, "dec_tile64_xcd%d%s", m, m == 64 ? " (product)" : "");
    report(name, time_ms(f), bad);
  }
  // ---- decode v5 (register-pipelined rows, 16-B column chunks): every column checked
  auto dec5 = [&](auto* k, int WG, int64_t xcd) {
    raise_lds_cap(k);
    const size_t lds = (size_t)64 * 848;
    const int64_t g = persistent_grid(k, lds, tiles, WG);
    FixedLaunch D = L;
    D.xcd_run = xcd < 0 ? (g % 8 == 0 ? g / 8 : 0) : xcd;
    return [=]() { hipLaunchKernelGGL(k, dim3((unsigned)g), dim3(WG), lds, 0, D, D.fields, rows, tiles, status); };
  };
  auto run_dec5 = [&](const char* name, auto* k, int WG, int64_t xcd = 0) {
    for (int c = 0; c < 104; ++c) CHECK(hipMemset(dcols[c], 0, n * width[c]));
    auto f = dec5(k, WG, xcd);
    f();
    CHECK(hipDeviceSynchronize());
    unsigned long long bad = 0;
    for (int c = 0; c < 104; ++c) bad += diff(cols[c], dcols[c], n * width[c]);
    report(name, time_ms(f), bad);
  };
  run_dec5("dec_v5_wg1024_k4_k3", &decode_fixed_v5_kernel<64, 1024, 4, 3, 0>, 1024);
  run_dec5("dec_v5_wg1024_k4_k3_xcd", &decode_fixed_v5_kernel<64, 1024, 4, 3, 0>, 1024, -1);
  run_dec5("dec_v5_wg1024_k4_k3_xcdblk", &decode_fixed_v5_kernel<64, 1024, 4, 3, 0>, 1024, T8);

  report("dec_tile64 dispatch order (again 2)", time_ms(base_dec), 0);
  run_dec5("dec_v5_wg1024_k4_k3 (again)", &decode_fixed_v5_kernel<64, 1024, 4, 3, 0>, 1024);
  run("enc_r64_wg1024_k3_xcd (product, again)", &encode_fixed_v5_kernel<64, 1024, 3, 0>, 64, 1024, -1);
  run("enc_r64_wg1024_k3_xcdblk (again)", &encode_fixed_v5_kernel<64, 1024, 3, 0>, 64, 1024, T8);
  report("dec_tile64 dispatch order (again)", time_ms(base_dec), 0);
  return 0;
}
