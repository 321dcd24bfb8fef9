// frames.hip — frame index of a self-delimiting STREAM batch on the device.
//
// A receiver on an RPC socket has only the frame stream that N calls of
// Encoder.encode(MemoryBuffer, T) wrote: [i32 size][i64 schemaHash][row] back
// to back, size = 8 + rowSize (Encoders.java:213-225). Encoder.decode(MemoryBuffer)
// walks it frame by frame — readInt32, readInt64 (hash check), row.pointTo,
// increaseReaderIndex(size - 8) (Encoders.java:176-193). That walk is serial;
// here it is split over chunks of the stream and stitched:
//
//  1. spec  (one lane per chunk): the first plausible frame start in the chunk
//     (4-byte aligned position whose next 8 bytes equal the schema hash and whose
//     size is sane) — chunk 0 starts at 0 — then the walk of sizes from it to the
//     first frame start at or past the chunk's end: (start, exit, frames).
//  2. check (one lane per chunk): chunk k is consistent when its start equals the
//     exit of chunk k-1 (then, by induction from chunk 0, its walk IS the true
//     chain); any inconsistency, or a chunk with no candidate, sets a flag.
//  3. fixup (one workgroup, only when flagged): Gauss-Seidel over contiguous
//     blocks of chunks — each chunk re-walks from its predecessor's exit — until
//     no exit changes. Payload bytes that mimic a frame header (hash + plausible
//     size) can mislead step 1 but not this step.
//  4. scan of the per-chunk frame counts -> frame index of each chunk's first frame.
//  5. write (one lane per chunk): row_offsets[f] = frame start (the positions
//     step 1 saved, or a re-walk for chunks the fix-up changed or with more than
//     kSaved frames), row_offsets[N] = end of frame N-1; a size out of range or
//     fewer than N frames in rows_bytes -> FORY_ERR_CORRUPT (frames past N are
//     never read).
// Schema hashes are checked by the decode kernels that follow (per frame), as in
// Encoders.decode; the walk itself follows sizes only.
#include "kcommon.h"

namespace fory_amd {

namespace {

constexpr int64_t kNone = -1;    // chunk holds no candidate frame start
constexpr int64_t kBroken = -2;  // the chain hit a size out of range
// Frame starts the spec walk saves per chunk (uint16 offsets from the chunk base,
// chunk <= 64 KiB), stored position-major (pos[j * chunks + k]) so the write pass
// reads them coalesced; chunks target ~20 frames.
constexpr int kSaved = 32;

// Frame header at p (4-byte aligned offset into the stream): size field and hash.
__device__ __forceinline__ uint32_t frame_size(const uint8_t* rows, int64_t p) {
  return *gp(reinterpret_cast<const uint32_t*>(rows + p));
}

// A size field that can start a frame of this plan: >= 8 + fixed_size, a multiple
// of 8 (rows are 8-byte padded) and the frame inside the stream.
__device__ __forceinline__ bool sane_size(uint32_t size, int64_t p, const FrameIndexLaunch& L) {
  return size >= (uint32_t)(8 + L.fixed_size) && (size & 7) == 0 && p + 4 + (int64_t)size <= L.rows_bytes;
}

// Walks sizes from p while p < end; returns the first position >= end (or
// kBroken) and the number of frames started before end.
// pos (nullable): the first kSaved frame starts, relative to `base`, at pos[j * stride].
__device__ __forceinline__ int64_t walk(const uint8_t* rows, int64_t p, int64_t end, const FrameIndexLaunch& L,
                                        int64_t* frames, uint16_t* pos = nullptr, int64_t base = 0,
                                        int64_t stride = 0) {
  int64_t f = 0;
  while (p < end) {
    const uint32_t size = frame_size(rows, p);
    if (!sane_size(size, p, L)) {
      *frames = f;
      return kBroken;
    }
    if (pos && f < kSaved) pos[f * stride] = (uint16_t)(p - base);
    ++f;
    p += 4 + (int64_t)size;
  }
  *frames = f;
  return p;
}

__global__ __launch_bounds__(kWG) void frame_spec_kernel(FrameIndexLaunch L, const uint8_t* __restrict__ rows,
                                                         int64_t* __restrict__ start, int64_t* __restrict__ exit_,
                                                         int64_t* __restrict__ count, uint16_t* __restrict__ pos,
                                                         int32_t* __restrict__ saved) {
  const int64_t k = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (k >= L.chunks) return;
  const int64_t base = k * L.chunk, end = min(base + L.chunk, L.rows_bytes);
  const uint32_t hlo = (uint32_t)(uint64_t)L.schema_hash, hhi = (uint32_t)((uint64_t)L.schema_hash >> 32);
  int64_t s = kNone;
  if (k == 0) {
    s = 0;
  } else {
    // S positions per step from S + 2 dwords, all loads of a step in flight at once
    // (the first frame start is on average half a frame into the chunk; S = 32 and
    // 8-frame chunks were not faster: Mixed index 0.94 / 1.05 ms vs 0.92 ms)
    constexpr int S = 8;
    const int64_t lim = L.rows_bytes - 12;  // a candidate needs its 12 header bytes
    auto ld = [&](int64_t q) -> uint32_t { return q + 4 <= L.rows_bytes ? frame_size(rows, q) : 0u; };
    for (int64_t p = base; p < end && p <= lim && s == kNone; p += 4 * S) {
      uint32_t d[S + 2];
#pragma unroll
      for (int j = 0; j < S + 2; ++j) d[j] = ld(p + 4 * j);
#pragma unroll
      for (int j = 0; j < S; ++j) {
        const int64_t q = p + 4 * j;
        if (s == kNone && q < end && q <= lim && d[j + 1] == hlo && d[j + 2] == hhi && sane_size(d[j], q, L)) s = q;
      }
    }
  }
  int64_t frames = 0, ex = kNone;
  if (s != kNone) ex = walk(rows, s, end, L, &frames, pos + k, base, L.chunks);
  start[k] = s;
  exit_[k] = ex;
  count[k] = frames;
  saved[k] = frames <= kSaved ? (int32_t)frames : -1;
}

// Chunk k's walk is the true chain iff its start is its predecessor's exit.
// Inconsistent chunks are marked dirty for the fix-up, which visits only those and
// the chunks whose entry it moves.
__global__ __launch_bounds__(kWG) void frame_check_kernel(FrameIndexLaunch L, const int64_t* __restrict__ start,
                                                          const int64_t* __restrict__ exit_, int64_t* flag,
                                                          uint8_t* __restrict__ dirty, int32_t* __restrict__ moved) {
  const int64_t k = (int64_t)blockIdx.x * kWG + threadIdx.x;
  if (k >= L.chunks) return;
  bool ok;
  if (k == 0) ok = true;
  else if (exit_[k - 1] == kBroken) ok = true;  // the chain ended before this chunk: nothing here counts
  else ok = start[k] != kNone && start[k] == exit_[k - 1];
  if (k > 0 && start[k - 1] == kNone) ok = false;  // a chunk without a candidate passes its entry through
  dirty[k] = ok ? 0 : 1;
  moved[k] = 0;
  if (!ok) atomicOr(reinterpret_cast<unsigned long long*>(flag), 1ull);
}

// One workgroup: chunk k's entry is chunk k-1's exit; a chunk whose start differs
// re-walks from its entry. Thread t owns chunks [t*B, (t+1)*B) and sweeps them in
// order (its own updates propagate at once); sweeps repeat until no exit changes,
// so after sweep i at least the blocks 0..i-1 hold the true chain.
// Only dirty chunks (check kernel) and chunks whose predecessor's exit moved are
// visited: a few inconsistent chunks (a frame longer than a chunk, a payload that
// mimics a header) cost a few walks, not a sweep over every chunk.
__global__ __launch_bounds__(1024) void frame_fixup_kernel(FrameIndexLaunch L, const uint8_t* __restrict__ rows,
                                                           int64_t* start, int64_t* exit_, int64_t* count,
                                                           int32_t* saved, const int64_t* flag, uint8_t* dirty,
                                                           int32_t* moved) {
  if (*flag == 0) return;
  __shared__ int changed;
  const int64_t B = (L.chunks + 1023) / 1024;
  const int64_t k0 = (int64_t)threadIdx.x * B, k1 = min(k0 + B, L.chunks);
  for (int64_t sweep = 0; sweep <= 1025; ++sweep) {
    if (threadIdx.x == 0) changed = 0;
    __syncthreads();
    bool mine = false;
    bool carry = false;  // this thread moved chunk k-1's exit
    for (int64_t k = k0; k < k1; ++k) {
      bool need = carry;
      carry = false;
      // the previous block's last chunk: acquire pairs with the release below, so a
      // seen flag comes with the exit_[k-1] stored before it
      if (k == k0 && k > 0)
        need = __hip_atomic_exchange(&moved[k - 1], 0, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != 0;
      if (dirty[k]) {
        need = true;
        dirty[k] = 0;
      }
      if (!need) continue;
      const int64_t entry = k == 0 ? 0 : __hip_atomic_load(&exit_[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int64_t base = k * L.chunk, end = min(base + L.chunk, L.rows_bytes);
      int64_t s, ex, frames = 0;
      if (entry == kBroken || entry == kNone) {
        s = kNone;
        ex = kBroken;
      } else if (entry >= end) {  // a frame spans the whole chunk
        s = kNone;
        ex = entry;
      } else {
        s = entry;
        if (s == start[k] && __hip_atomic_load(&exit_[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != kNone)
          continue;  // already walked from here
        ex = walk(rows, s, end, L, &frames);
      }
      if (s != start[k] || ex != __hip_atomic_load(&exit_[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ||
          frames != count[k]) {
        start[k] = s;
        count[k] = frames;
        saved[k] = -1;  // the positions step 1 saved are not this chain's: the write pass re-walks
        __hip_atomic_store(&exit_[k], ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        mine = true;
        // the next block's first chunk re-checks: release orders the exit_ store first
        if (k + 1 == k1) __hip_atomic_exchange(&moved[k], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        else carry = true;
      }
    }
    __threadfence();
    if (mine) changed = 1;
    __syncthreads();
    if (!changed) break;
    __syncthreads();
  }
}

// Chunk k's frames get indices base[k] .. base[k] + count[k] - 1 (count scanned in place),
// with the stores coalesced (round 6): a workgroup per kWG chunks stages their first frame
// indices, counts and saved positions in LDS, then its threads write consecutive offs[f] --
// each finds its chunk by a binary search over the staged frame bases -- where round 5's
// write pass had each lane store its own chunk's ~16 offsets at a 128-byte stride from the
// next lane's (64 partial lines per store instruction). Chunks
// whose positions were not all saved (a fix-up re-walk, > kSaved frames) are walked by
// their own thread as before.
__global__ __launch_bounds__(kWG) void frame_write_co_kernel(FrameIndexLaunch L, const uint8_t* __restrict__ rows,
                                                             const int64_t* __restrict__ start,
                                                             const int64_t* __restrict__ exit_,
                                                             const int64_t* __restrict__ base,
                                                             const uint16_t* __restrict__ pos,
                                                             const int32_t* __restrict__ saved,
                                                             int64_t* __restrict__ offs, int32_t* status) {
  __shared__ int64_t fb[kWG + 1];        // first frame index of each chunk (+ the end)
  __shared__ uint8_t ok[kWG];            // its frames' positions are all saved
  __shared__ uint16_t sp[kSaved][kWG];   // the saved positions, position-major
  const int t = threadIdx.x;
  const int64_t k0 = (int64_t)blockIdx.x * kWG;
  const int nk = L.chunks - k0 < kWG ? (int)(L.chunks - k0) : kWG;
  const int64_t k = k0 + t;
  if (k == 0 && base[L.chunks] < L.num_rows) set_status(status, FORY_ERR_CORRUPT);  // fewer than N frames
  int64_t f = 0, cnt = 0, p = -1;
  bool sv = false;
  if (t < nk) {
    f = base[k];
    cnt = base[k + 1] - f;
    p = start[k];
    sv = p >= 0 && saved[k] == cnt;
#pragma unroll 8
    for (int j = 0; j < kSaved; ++j) sp[j][t] = pos[j * L.chunks + k];
    fb[t] = f;
    ok[t] = sv ? 1 : 0;
    if (t == nk - 1) fb[nk] = base[k + 1];
  }
  __syncthreads();
  if (t < nk && p >= 0 && f < L.num_rows) {
    const int64_t cbase = k * L.chunk, end = min(cbase + L.chunk, L.rows_bytes);
    if (sv) {
      // the chain broke inside this chunk before frame N: Encoders.decode would read past it
      if (exit_[k] == kBroken && f + cnt < L.num_rows) set_status(status, FORY_ERR_CORRUPT);
    } else {
      int64_t g = f;
      while (p < end && g < L.num_rows) {
        const uint32_t size = frame_size(rows, p);
        if (!sane_size(size, p, L)) {  // Encoders.decode would read past the frame: corrupt stream
          set_status(status, FORY_ERR_CORRUPT);
          break;
        }
        offs[g] = p;
        p += 4 + (int64_t)size;
        if (g == L.num_rows - 1) offs[L.num_rows] = p;
        ++g;
      }
    }
  }
  // the saved chunks' frames: consecutive threads, consecutive offsets
  const int64_t F0 = fb[0], F1 = min(fb[nk], L.num_rows);
  for (int64_t g = F0 + t; g < F1; g += kWG) {
    int a = 0, b = nk - 1;  // the last chunk whose first frame is at or before g
    while (a < b) {
      const int mid = (a + b + 1) >> 1;
      if (fb[mid] <= g) a = mid;
      else b = mid - 1;
    }
    if (!ok[a]) continue;
    const int64_t q = (k0 + a) * L.chunk + sp[g - fb[a]][a];
    offs[g] = q;
    if (g == L.num_rows - 1) offs[L.num_rows] = q + 4 + (int64_t)frame_size(rows, q);
  }
}

}  // namespace

void frame_index_plan(int64_t num_rows, int64_t rows_bytes, int32_t idx_frames, int64_t* chunk, int64_t* chunks) {
  // ~20 frames per chunk at the batch's mean frame size, in [1, 64] KiB (the plan's
  // FORY_ROWFMT_IDXFRAMES knob overrides the 20, for A/B). Round 6, three alternating
  // rounds on one box (profiles/r06/idxframes/): index 0.78 -> 0.70-0.73 ms (Mixed 16Mi),
  // 0.336 -> 0.317 ms (Nested 8Mi) against 16; 24 was between them.
  const int64_t n = num_rows > 0 ? num_rows : 1;
  const int64_t per = idx_frames > 0 ? idx_frames : 20;
  int64_t c = (per * (rows_bytes / n) + 255) / 256 * 256;
  c = c < 1024 ? 1024 : (c > 65536 ? 65536 : c);
  *chunk = c;
  *chunks = rows_bytes > 0 ? (rows_bytes + c - 1) / c : 0;
}

int64_t frame_index_words(int64_t num_rows, int64_t rows_bytes, int32_t idx_frames) {
  int64_t c, k;
  frame_index_plan(num_rows, rows_bytes, idx_frames, &c, &k);
  // start, exit, count (+ total), flag, scan partials, saved counts (int32), positions
  // (uint16), moved flags (int32), dirty flags (uint8)
  return 3 * k + 2 + 2 + scan_partials(k) + (k + 1) / 2 + (kSaved * k + 3) / 4 + 1 + (k + 1) / 2 + (k + 7) / 8 + 1;
}

hipError_t launch_frame_index(const FrameIndexLaunch& L0, const uint8_t* rows, int64_t* offs, int64_t* ws,
                              int32_t* status, hipStream_t s) {
  FrameIndexLaunch L = L0;
  frame_index_plan(L.num_rows, L.rows_bytes, L.idx_frames, &L.chunk, &L.chunks);
  if (L.num_rows <= 0) {
    (void)hipMemsetAsync(offs, 0, sizeof(int64_t), s);
    return hipGetLastError();
  }
  const int64_t K = L.chunks;
  int64_t* start = ws;
  int64_t* exit_ = start + K;
  int64_t* count = exit_ + K;  // K + 1 (scan total)
  int64_t* flag = count + K + 1;
  int64_t* partials = flag + 2;
  int32_t* saved = reinterpret_cast<int32_t*>(partials + scan_partials(K));
  uint16_t* pos = reinterpret_cast<uint16_t*>(saved + 2 * ((K + 1) / 2));
  int32_t* moved = reinterpret_cast<int32_t*>(pos + 4 * ((kSaved * K + 3) / 4) + 4);
  uint8_t* dirty = reinterpret_cast<uint8_t*>(moved + 2 * ((K + 1) / 2));
  (void)hipMemsetAsync(flag, 0, sizeof(int64_t), s);
  const unsigned blocks = (unsigned)((K + kWG - 1) / kWG);
  hipLaunchKernelGGL(frame_spec_kernel, dim3(blocks), dim3(kWG), 0, s, L, rows, start, exit_, count, pos, saved);
  hipLaunchKernelGGL(frame_check_kernel, dim3(blocks), dim3(kWG), 0, s, L, start, exit_, flag, dirty, moved);
  hipLaunchKernelGGL(frame_fixup_kernel, dim3(1), dim3(1024), 0, s, L, rows, start, exit_, count, saved, flag, dirty,
                     moved);
  hipError_t e = launch_scan_i64(count, K, partials, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(frame_write_co_kernel, dim3(blocks), dim3(kWG), 0, s, L, rows, start, exit_, count, pos, saved,
                     offs, status);
  return hipGetLastError();
}

}  // namespace fory_amd
