// capi.cpp — the extern "C" boundary (include/fory_rowfmt.h).
//
// Host-side glue only: validate arguments the way the reference validates
// them (Preconditions / bounds checks / schema-hash check), bind the
// caller's columns into a device table in the caller's workspace, and
// enqueue the kernels of kernels.hip on the caller's stream.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <atomic>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/fory_rowfmt.h"
#include "kernels.h"
#include "plan.h"

using fory_amd::ColumnDev;
using fory_amd::FixedFieldDev;
using fory_amd::Plan;

// Columnar tree engine layout of a plan (treecol.hip): var nodes by depth.
struct TcInfo {
  bool ok = false;                  // generic plan of <= kTcMaxNodes nodes
  std::vector<fory_amd::TcVar> var;  // by depth, pre-order within a depth
  std::vector<int32_t> vidx;        // node -> var index (-1: scalar)
  std::vector<int32_t> parent;      // node -> parent node (-1: the row)
};

struct fory_plan {
  Plan p;
  TcInfo tc;
  uint64_t id = 0;  // unique per plan_create (the encode memo's key; addresses are reused)
};

namespace fory_amd {
bool fixed_tiled_supported(int stride);
}

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

int hip_fail(hipError_t e, const char* what) {
  return fail(FORY_ERR_DEVICE, std::string(what) + ": " + hipGetErrorString(e));
}

constexpr int64_t kAlign = 256;
int64_t align_up(int64_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

int64_t table_bytes(const Plan& p) {
  // fixed-width: the width-ordered field table
  if (p.fixed_width)  // then the per-slot validity pointers (nullable v5 kernels)
    return align_up((int64_t)p.top.size() * (int64_t)sizeof(FixedFieldDev)) + align_up((int64_t)p.top.size() * 8);
  if (p.generic)  // columns, then the node table
    return align_up((int64_t)p.nodes.size() * (int64_t)sizeof(ColumnDev)) +
           align_up((int64_t)p.gnodes.size() * (int64_t)sizeof(fory_amd::GNode));
  return align_up((int64_t)p.nodes.size() * (int64_t)sizeof(ColumnDev)) +
         align_up((int64_t)p.program.size() * (int64_t)sizeof(fory_amd::Op)) +
         align_up((int64_t)p.program.size() * (int64_t)sizeof(fory_amd::VarFieldDev)) +
         align_up((int64_t)p.program.size() * (int64_t)sizeof(FixedFieldDev)) +
         align_up((int64_t)p.program.size() * (int64_t)sizeof(fory_amd::StructDev));
}

// STRING/BINARY/LIST fields at any struct level (the tile kernels' var fields).
int64_t num_var_ops(const Plan& p) {
  int64_t n = 0;
  for (const fory_amd::Op& op : p.program)
    if (op.code == fory_amd::OP_BYTES || op.code == fory_amd::OP_LIST) ++n;
  return n;
}

bool use_tiled(const Plan& p, int frame) {
  return p.fixed_width && fory_amd::fixed_tiled_supported(p.fixed_size + fory_amd::frame_header_bytes(frame));
}

void tc_forget(const void* ws);
void td_forget(const void* ws);

// Workspace memos of the columnar engine: encode may reuse the sizes its encoded_size
// left in the workspace (KEEP_TC), decode_sizes the positions of the levels the previous
// decode_sizes ran (KEEP_TD); every other call may overwrite them.
enum { KEEP_NONE = 0, KEEP_TC = 1, KEEP_TD = 2 };
int check_common(const fory_plan* plan, const fory_column* cols, int64_t n, int frame,
                 void* ws, int64_t ws_bytes, int keep_memo = KEEP_NONE) {
  if (keep_memo != KEEP_TC) tc_forget(ws);
  if (keep_memo != KEEP_TD) td_forget(ws);
  if (!plan) return fail(FORY_ERR_INVALID_ARGUMENT, "plan is null");
  if (n < 0) return fail(FORY_ERR_INVALID_ARGUMENT, "num_rows < 0");
  if (frame != FORY_FRAME_RAW && frame != FORY_FRAME_STREAM && frame != FORY_FRAME_COLLECTION &&
      frame != FORY_FRAME_HASHED)
    return fail(FORY_ERR_INVALID_ARGUMENT,
                "frame_mode must be 0 (raw), 1 (stream), 2 (collection) or 3 (hashed)");
  if (frame == FORY_FRAME_COLLECTION) {
    const Plan& p = plan->p;
    const int k = p.top.size() == 1 ? p.nodes[p.top[0]].kind : -1;
    if (k != fory_amd::KIND_LIST && k != fory_amd::KIND_MAP)
      return fail(FORY_ERR_INVALID_ARGUMENT,
                  "collection frames need a plan of exactly one list or map field (ArrayEncoder / MapEncoder)");
  }
  if (n > 0 && !cols) return fail(FORY_ERR_INVALID_ARGUMENT, "cols is null");
  const int64_t need = fory_rowfmt_workspace_bytes(plan, n);
  if (n > 0 && (!ws || ws_bytes < need))
    return fail(FORY_ERR_INVALID_ARGUMENT,
                "workspace too small: need " + std::to_string(need) + " bytes");
  return FORY_OK;
}

// Binds the top-level columns of a fixed-width plan (encode: inputs; decode: outputs).
int bind_fixed(const Plan& p, const fory_column* cols, int64_t n, bool decode,
               std::vector<FixedFieldDev>* out) {
  out->resize(p.top.size());
  for (size_t k = 0; k < p.top.size(); ++k) {
    const int32_t idx = p.top[k];
    const fory_amd::Node& nd = p.nodes[idx];
    const fory_column& c = cols[idx];
    if (n > 0 && !c.values)
      return fail(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(idx) + " has no values");
    if (n > 0 && c.length < n)
      return fail(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(idx) + " shorter than num_rows");
    if (decode && n > 0 && c.capacity > 0 && c.capacity < n * nd.width)
      return fail(FORY_ERR_CAPACITY, "column " + std::to_string(idx) + " capacity too small");
    FixedFieldDev f{};
    f.width = nd.width;
    f.flags = (nd.nullable ? 1 : 0) | (nd.kind == fory_amd::KIND_BOOL ? 2 : 0);
    if (decode) {
      f.out_values = static_cast<uint8_t*>(c.values);
      f.out_validity = nd.nullable ? c.validity : nullptr;
    } else {
      f.values = static_cast<const uint8_t*>(c.values);
      f.validity = nd.nullable ? c.validity : nullptr;
    }
    f.slot = (int32_t)k;
    (*out)[k] = f;
  }
  // width groups 8, 4, 2, 1 (stable): see FixedFieldDev
  std::stable_sort(out->begin(), out->end(),
                   [](const FixedFieldDev& a, const FixedFieldDev& b) { return a.width > b.width; });
  return FORY_OK;
}

// String/binary list elements and map keys/values: their columns are indexed by
// element, so decode sizes them in a second lengths pass (decode_sizes).
std::vector<int32_t> elem_bytes_cols(const Plan& p) {
  std::vector<int32_t> out;
  for (const fory_amd::Op& op : p.program) {
    if (op.code == fory_amd::OP_LIST && ((op.e >> 8) & 4)) out.push_back(op.c);
    if (op.code == fory_amd::OP_MAP) {
      if ((op.e >> 16) & 4) out.push_back(op.c);
      if ((op.e >> 24) & 4) out.push_back(op.c + 1);
    }
  }
  return out;
}

// sizes_pass: element string/binary columns may come without offsets (decode_sizes
// before the caller knows the element count).
int bind_var(const Plan& p, const fory_column* cols, int64_t n, std::vector<ColumnDev>* out,
             bool sizes_pass = false) {
  std::vector<int32_t> elem = sizes_pass ? elem_bytes_cols(p) : std::vector<int32_t>();
  out->resize(p.nodes.size());
  for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
    const fory_amd::Node& nd = p.nodes[idx];
    const fory_column& c = cols[idx];
    ColumnDev d{};
    d.values = static_cast<const uint8_t*>(c.values);
    d.offsets = c.offsets;
    d.validity = nd.nullable ? c.validity : nullptr;
    d.out_values = static_cast<uint8_t*>(c.values);
    d.out_offsets = c.offsets;
    d.out_validity = nd.nullable ? c.validity : nullptr;
    if (n > 0) {
      if ((nd.kind == fory_amd::KIND_BYTES || nd.kind == fory_amd::KIND_LIST || nd.kind == fory_amd::KIND_MAP) &&
          !c.offsets && std::find(elem.begin(), elem.end(), (int32_t)idx) == elem.end())
        return fail(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(idx) + " needs offsets");
    }
    (*out)[idx] = d;
  }
  return FORY_OK;
}

// Plan tables reach the workspace by an async copy from pinned host memory that
// outlives the call: per device a pool of pinned slots (process lifetime). A slot is
// taken only when the copy that last read it has completed (hipEventQuery: nobody
// waits under a lock); when every slot is still in flight the pool grows, up to
// kMaxSlots, and only then the oldest slot is waited for — outside the lock. A copy
// straight from a local vector could be read by the DMA engine after the call
// returned (a flaky plan table in the host pipeline, round 1).
struct UploadSlot {
  void* buf = nullptr;
  size_t cap = 0;
  hipEvent_t ev = nullptr;
  hipStream_t st = nullptr;  // the stream the slot's last copy was queued on
  uint64_t stamp = 0;        // queue order of that copy
  bool pending = false;      // a copy was queued and not yet seen complete
  bool busy = false;         // taken by a call right now
  bool dead = false;         // its event reported an error: never reused (its copy may still read it)
};

struct UploadRing {
  static constexpr size_t kMaxSlots = 256;
  std::mutex mu;
  std::vector<UploadSlot*> slots;  // never freed (process lifetime)
  uint64_t clock = 0;
};

std::mutex g_rings_mu;
std::map<int, UploadRing*>* g_rings = new std::map<int, UploadRing*>();  // never freed

// hipEventQuery: true when the slot's copy is done (clears the "not ready" status it
// leaves as the thread's last error, so a caller's hipGetLastError is not disturbed).
// Only hipSuccess frees the slot. Any other answer (a sticky fault of the device, a
// destroyed stream) says nothing about whether the DMA engine still reads the slot's
// buffer, so the slot is retired for good -- round 5 treated every non-"not ready"
// answer as completion and could hand a buffer to the next table while a copy still
// read it. The error itself reaches the caller through its next
// synchronising call.
bool slot_done(UploadSlot* sl) {
  if (sl->dead) return false;
  if (!sl->pending) return true;
  const hipError_t e = hipEventQuery(sl->ev);
  if (e == hipSuccess) {
    sl->pending = false;
    return true;
  }
  (void)hipGetLastError();
  if (e != hipErrorNotReady) sl->dead = true;
  return false;
}

int upload(void* ws, const void* host, int64_t bytes, hipStream_t s) {
  if (bytes == 0) return FORY_OK;
  int dev = 0;
  (void)hipGetDevice(&dev);
  UploadRing* r = nullptr;
  {
    std::lock_guard<std::mutex> lock(g_rings_mu);
    UploadRing*& rp = (*g_rings)[dev];
    if (!rp) rp = new UploadRing();
    r = rp;
  }
  UploadSlot* sl = nullptr;
  bool wait_first = false;
  {
    std::lock_guard<std::mutex> lock(r->mu);
    UploadSlot* oldest = nullptr;
    for (UploadSlot* c : r->slots) {
      if (c->busy || c->dead) continue;
      if (slot_done(c)) {
        if (!sl || (sl->cap < (size_t)bytes && c->cap >= (size_t)bytes)) sl = c;
        if (sl->cap >= (size_t)bytes) break;
      } else if (!oldest || c->stamp < oldest->stamp) {
        oldest = c;
      }
    }
    if (!sl && r->slots.size() < UploadRing::kMaxSlots) {
      sl = new UploadSlot();
      r->slots.push_back(sl);
    }
    if (!sl) sl = oldest, wait_first = true;
    if (!sl) return fail(FORY_ERR_DEVICE, "plan table staging: every slot is taken");
    sl->busy = true;
  }
  hipError_t e = hipSuccess;
  if (wait_first) e = hipEventSynchronize(sl->ev);  // the oldest copy, outside the lock
  if (e == hipSuccess && !sl->ev) e = hipEventCreateWithFlags(&sl->ev, hipEventDisableTiming);
  if (e == hipSuccess && sl->cap < (size_t)bytes) {
    if (sl->buf) (void)hipHostFree(sl->buf);
    sl->buf = nullptr;
    sl->cap = 0;
    const size_t want = std::max<size_t>((size_t)bytes, 64 * 1024);
    e = hipHostMalloc(&sl->buf, want, hipHostMallocPortable | hipHostMallocCoherent);
    if (e == hipSuccess) sl->cap = want;
  }
  bool queued = false;
  if (e == hipSuccess) {
    std::memcpy(sl->buf, host, (size_t)bytes);
    e = hipMemcpyAsync(ws, sl->buf, (size_t)bytes, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = hipEventRecord(sl->ev, s), queued = true;
  }
  {
    std::lock_guard<std::mutex> lock(r->mu);
    if (queued || wait_first) sl->pending = queued;
    if (wait_first && !queued && e != hipSuccess) sl->dead = true;  // its old copy's fate is unknown
    sl->st = s;
    sl->stamp = ++r->clock;
    sl->busy = false;
  }
  if (e != hipSuccess) return hip_fail(e, "plan table upload");
  return FORY_OK;
}

// The field table, then per slot (schema ordinal) the column's validity pointer (input on
// encode, output on decode; null for not-null fields and absent validity), one upload.
// *valid8: every such pointer is 8-byte aligned (the nullable v5 kernels' word accesses).
int upload_fixed_tables(const Plan& p, void* ws, const std::vector<FixedFieldDev>& tab, bool decode, hipStream_t s,
                        int32_t* valid8) {
  const int64_t nf = (int64_t)tab.size();
  const int64_t t0 = align_up(nf * (int64_t)sizeof(FixedFieldDev));
  std::vector<uint8_t> buf((size_t)(t0 + nf * 8), 0);
  std::memcpy(buf.data(), tab.data(), (size_t)nf * sizeof(FixedFieldDev));
  *valid8 = 1;
  for (const FixedFieldDev& f : tab) {
    const uint8_t* v = decode ? f.out_validity : f.validity;
    if (!(f.flags & 1)) v = nullptr;
    if (v && (reinterpret_cast<uintptr_t>(v) & 7)) *valid8 = 0;
    std::memcpy(buf.data() + t0 + 8 * f.slot, &v, 8);
  }
  (void)p;
  return upload(ws, buf.data(), (int64_t)buf.size(), s);
}

fory_amd::FixedLaunch fixed_launch(const Plan& p, const void* table, int64_t n, int frame) {
  fory_amd::FixedLaunch L{};
  L.fields = static_cast<const FixedFieldDev*>(table);
  L.num_fields = (int32_t)p.top.size();
  L.slot_validity = reinterpret_cast<const uint8_t* const*>(
      static_cast<const uint8_t*>(table) + align_up((int64_t)p.top.size() * (int64_t)sizeof(FixedFieldDev)));
  L.bitmap_bytes = p.bitmap_bytes;
  L.fixed_size = p.fixed_size;
  L.stride = p.fixed_size + fory_amd::frame_header_bytes(frame);
  {  // v5's per-lane record order (LDS bank spread), from the row layout
    const int hdr = fory_amd::frame_header_bytes(frame), hdr_bm = hdr + p.bitmap_bytes;
    L.rot4 = fory_amd::v5_rotation(L.stride, hdr, hdr_bm, 4, false);
    L.rot8 = fory_amd::v5_rotation(L.stride, hdr, hdr_bm, 8, false);
    // the decode only for nullable plans: rotated reads cost the not-null raw decode 2 %
    // (15.73 vs 15.42 ms at 64Mi Struct104 rows) and gave the nullable one 3.5 % (4.30 vs
    // 4.46 ms at 16Mi boxed rows), alternating on one box (profiles/r05/rotation/)
    L.drot4 = p.any_nullable ? fory_amd::v5_rotation(L.stride, hdr, hdr_bm, 4, true) : 31;
    L.drot8 = p.any_nullable ? fory_amd::v5_rotation(L.stride, hdr, hdr_bm, 8, true) : 31;
  }
  L.schema_hash = p.schema_hash;
  L.num_rows = n;
  L.any_nullable = p.any_nullable ? 1 : 0;
  L.frame = frame;
  // width-group boundaries of the sorted table (bind_fixed)
  const int widths[4] = {8, 4, 2, 1};
  int at = 0;
  for (int g = 0; g < 4; ++g) {
    L.group[g] = at;
    for (int32_t t : p.top)
      if (p.nodes[t].width == widths[g]) ++at;
  }
  L.group[4] = at;
  return L;
}

int32_t* spill_ptr(const Plan& p, void* ws, int64_t n);

// LDS budget of one 64-record tile image for the varlen tile engine: 64 x an
// estimated row (fixed part, nested struct rows, ~32 bytes per string,
// ~16 elements per list), in [8, 64] KiB; small enough to keep several
// workgroups per CU. Bigger tiles spill to a second launch with a 96 KiB
// image (kSpillCap); FORY_ROWFMT_VARCAP overrides.
int var_tile_cap(const Plan& p, int frame) {
  int64_t est = p.fixed_size + fory_amd::frame_header_bytes(frame);
  for (size_t k = 0; k < p.nodes.size(); ++k) {
    const fory_amd::Node& nd = p.nodes[k];
    if (nd.kind == fory_amd::KIND_BYTES) est += 32;
    else if (nd.kind == fory_amd::KIND_LIST) est += 16 + 16 * std::max<int64_t>(1, p.nodes[nd.children[0]].width);
    else if (nd.kind == fory_amd::KIND_MAP)  // [i64][keys][values], ~16 entries
      est += 40 + 16 * (p.nodes[nd.children[0]].width + p.nodes[nd.children[1]].width);
    else if (nd.kind == fory_amd::KIND_STRUCT)  // child rows live in the variable region
      est += ((int64_t)(nd.children.size() + 63) / 64) * 8 + 8 * (int64_t)nd.children.size();
  }
  int64_t cap = (64 * est + 1023) / 1024 * 1024;
  return (int)std::min<int64_t>(std::max<int64_t>(cap, 8 * 1024), 64 * 1024);
}

// Var launch: columns table then program in the workspace.
int prepare_var(const Plan& p, const fory_column* cols, int64_t n, int frame, void* ws,
                hipStream_t s, fory_amd::VarLaunch* L, bool sizes_pass = false) {
  std::vector<ColumnDev> cd;
  int rc = bind_var(p, cols, n, &cd, sizes_pass);
  if (rc) return rc;
  const int64_t col_bytes = align_up((int64_t)cd.size() * (int64_t)sizeof(ColumnDev));
  const int64_t prog_bytes = align_up((int64_t)p.program.size() * (int64_t)sizeof(fory_amd::Op));
  const int64_t idx_bytes = align_up((int64_t)p.program.size() * (int64_t)sizeof(fory_amd::VarFieldDev));
  const int64_t fix_bytes = align_up((int64_t)p.program.size() * (int64_t)sizeof(FixedFieldDev));
  // tile kernels: var-field descriptors (program order), the width-sorted
  // fixed-field table and the struct table, each field tagged with its
  // enclosing struct (0 = the row)
  std::vector<fory_amd::VarFieldDev> var;
  std::vector<FixedFieldDev> fix;
  std::vector<fory_amd::StructDev> st;
  std::vector<int32_t> stack{0};
  for (size_t k = 0; k < p.program.size(); ++k) {
    const fory_amd::Op& op = p.program[k];
    const int32_t parent = stack.back();
    if (op.code == fory_amd::OP_STRUCT_BEGIN) {
      const fory_column& c = cols[op.b];
      fory_amd::StructDev sd{};
      sd.validity = (op.d & 1) ? c.validity : nullptr;
      sd.out_validity = (op.d & 1) ? c.validity : nullptr;
      sd.parent = parent;
      sd.slot = op.a;
      sd.nfields = op.c;
      sd.hdr = (int32_t)(((op.c + 63) / 64) * 8);
      sd.flags = op.d;
      st.push_back(sd);
      stack.push_back((int32_t)st.size());
    } else if (op.code == fory_amd::OP_STRUCT_END) {
      stack.pop_back();
    } else if (op.code == fory_amd::OP_FIXED) {
      const fory_column& c = cols[op.b];
      FixedFieldDev f{};
      f.values = static_cast<const uint8_t*>(c.values);
      f.out_values = static_cast<uint8_t*>(c.values);
      f.validity = (op.d & 1) ? c.validity : nullptr;
      f.out_validity = (op.d & 1) ? c.validity : nullptr;
      f.width = op.c;
      f.flags = op.d;
      f.slot = op.a;
      f.parent = parent;
      fix.push_back(f);
    } else if (op.code == fory_amd::OP_BYTES || op.code == fory_amd::OP_LIST) {
      const fory_column& c = cols[op.b];
      fory_amd::VarFieldDev v{};
      v.offsets = c.offsets;
      v.out_offsets = c.offsets;
      v.validity = (op.d & 1) ? c.validity : nullptr;
      v.out_validity = (op.d & 1) ? c.validity : nullptr;
      v.slot = op.a;
      v.flags = op.d;
      v.parent = parent;
      if (op.code == fory_amd::OP_LIST) {
        const fory_column& it = cols[op.c];
        v.is_list = 1;
        v.w = op.e & 0xff;
        v.iflags = op.e >> 8;
        v.values = static_cast<const uint8_t*>(it.values);
        v.out_values = static_cast<uint8_t*>(it.values);
        v.item_validity = (v.iflags & 1) ? it.validity : nullptr;
        v.out_item_validity = (v.iflags & 1) ? it.validity : nullptr;
      } else {
        v.w = 1;
        v.values = static_cast<const uint8_t*>(c.values);
        v.out_values = static_cast<uint8_t*>(c.values);
      }
      var.push_back(v);
    }
  }
  std::stable_sort(fix.begin(), fix.end(),
                   [](const FixedFieldDev& a, const FixedFieldDev& b) { return a.width > b.width; });
  std::vector<uint8_t> host((size_t)table_bytes(p), 0);
  const int64_t o_var = col_bytes + prog_bytes, o_fix = o_var + idx_bytes, o_st = o_fix + fix_bytes;
  std::memcpy(host.data(), cd.data(), cd.size() * sizeof(ColumnDev));
  std::memcpy(host.data() + col_bytes, p.program.data(), p.program.size() * sizeof(fory_amd::Op));
  std::memcpy(host.data() + o_var, var.data(), var.size() * sizeof(fory_amd::VarFieldDev));
  std::memcpy(host.data() + o_fix, fix.data(), fix.size() * sizeof(FixedFieldDev));
  std::memcpy(host.data() + o_st, st.data(), st.size() * sizeof(fory_amd::StructDev));
  rc = upload(ws, host.data(), (int64_t)host.size(), s);
  if (rc) return rc;
  uint8_t* wsb = static_cast<uint8_t*>(ws);
  bool has_map = false;  // (and lists of structs)
  for (const fory_amd::Op& op : p.program)
    has_map |= op.code == fory_amd::OP_MAP || op.code == fory_amd::OP_LIST_STRUCT ||
               (op.code == fory_amd::OP_LIST && ((op.e >> 8) & 4));
  // maps, lists of structs and lists of strings run on the generic tile interpreter
  // (enc_record / dec_record)
  L->flat = !has_map && frame != FORY_FRAME_COLLECTION && var.size() <= 32 &&
                    st.size() <= (size_t)fory_amd::kMaxTileStructs
                ? 1
                : 0;
  L->num_var = (int32_t)var.size();
  L->num_struct = (int32_t)st.size();
  L->vf = reinterpret_cast<const fory_amd::VarFieldDev*>(wsb + o_var);
  L->fix = reinterpret_cast<const FixedFieldDev*>(wsb + o_fix);
  L->st = reinterpret_cast<const fory_amd::StructDev*>(wsb + o_st);
  {
    const int widths[4] = {8, 4, 2, 1};
    int at = 0;
    for (int g = 0; g < 4; ++g) {
      L->fix_group[g] = at;
      for (const FixedFieldDev& f : fix)
        if (f.width == widths[g]) ++at;
    }
    L->fix_group[4] = at;
  }
  L->kn = p.kn;
  L->prof = fory_amd::var_prof_buffer((n + 63) / 64, p.kn.prof != 0);
  L->spill_count = spill_ptr(p, ws, n);
  L->spill = L->spill_count + 4;
  L->stg_bytes = p.kn.var_stg > 0 ? std::max(256, std::min(16384, p.kn.var_stg)) & ~15 : 2048;
  int64_t nested_fixed = 0;
  for (const fory_amd::StructDev& sd : st) nested_fixed += sd.hdr + 8LL * sd.nfields;
  for (const fory_amd::VarFieldDev& v : var) nested_fixed += v.is_list ? 8 : 0;
  L->nested_fixed = (int32_t)nested_fixed;
  int32_t est = 0;  // ~32 B per string, 16 items (+ their validity bits) per list
  for (const fory_amd::VarFieldDev& v : var) est = std::max(est, v.is_list ? 16 * v.w + 2 : 32);
  L->var_est_row = est;
  L->iv_split = var.size() == 1 && var[0].is_list && var[0].out_item_validity ? 1 : 0;
  L->nullable = 0;
  for (const FixedFieldDev& f : fix) L->nullable |= f.validity ? 1 : 0;
  for (const fory_amd::VarFieldDev& v : var) L->nullable |= v.validity ? 2 : 0;
  L->num_list = 0;
  L->list_mask = 0;
  L->bool_items = 0;
  for (size_t v = 0; v < var.size(); ++v)
    if (var[v].is_list) {
      ++L->num_list;
      if (v < 32) L->list_mask |= 1u << v;
      if (var[v].iflags & 2) L->bool_items = 1;
    }
  for (size_t k = 0; k < st.size() && k < (size_t)fory_amd::kMaxTileStructs; ++k) L->st_hdr[k] = st[k].hdr;
  L->cols = static_cast<const ColumnDev*>(ws);
  L->prog = reinterpret_cast<const fory_amd::Op*>(static_cast<uint8_t*>(ws) + col_bytes);
  L->num_ops = (int32_t)p.program.size();
  L->num_top = (int32_t)p.top.size();
  L->bitmap_bytes = p.bitmap_bytes;
  L->fixed_size = p.fixed_size;
  L->schema_hash = p.schema_hash;
  L->num_rows = n;
  L->frame = frame;
  L->tile_cap = var_tile_cap(p, frame);
  L->level2 = 0;
  return FORY_OK;
}

// Mean row/frame bytes of a decode batch, for the tile image size of the flat decode
// kernels (fit_cap), estimated from the output capacities the caller sized from
// decode_sizes (string bytes, list items): fixed part + child rows + per var field
// its mean payload and padding. No device read. 0 (static estimate) when a capacity
// is missing or the batch is small.
int64_t decode_mean_row(const Plan& p, const fory_amd::VarLaunch& L, const fory_column* cols, int64_t n, int frame) {
  if (!L.flat || n < 4096 || !cols) return 0;
  double row = p.fixed_size + fory_amd::frame_header_bytes(frame);
  for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
    const fory_amd::Node& nd = p.nodes[idx];
    if (nd.kind == fory_amd::KIND_STRUCT) {
      row += ((nd.children.size() + 63) / 64) * 8.0 + 8.0 * nd.children.size();
    } else if (nd.kind == fory_amd::KIND_BYTES) {
      if (cols[idx].capacity <= 0) return 0;
      row += (double)cols[idx].capacity / n + 3.5;  // + mean zero padding to 8
    } else if (nd.kind == fory_amd::KIND_LIST) {
      const int32_t item = nd.children[0];
      const int w = p.nodes[item].width > 0 ? p.nodes[item].width : 8;
      if (cols[item].capacity <= 0) return 0;
      const double items = (double)cols[item].capacity / w / n;
      row += 8 + 8.0 * ((int64_t)items / 64 + 1) + items * w + 3.5;
    }
  }
  return (int64_t)row;
}

int64_t* partials_ptr(const Plan& p, void* ws) {
  return reinterpret_cast<int64_t*>(static_cast<uint8_t*>(ws) + table_bytes(p));
}

// Scan partials: one scan over the rows, or the flat decode's tile-total scans of
// every var field at once.
int64_t partials_bytes(const Plan& p, int64_t n) {
  return align_up(std::max(fory_amd::scan_partials(n) + 2,
                           fory_amd::scan_multi_partials((n + 63) / 64, (int)num_var_ops(p))) * 8);
}

// Per-tile payload totals of the flat decode (after the scan partials).
int64_t* tile_totals_ptr(const Plan& p, void* ws, int64_t n) {
  return reinterpret_cast<int64_t*>(static_cast<uint8_t*>(ws) + table_bytes(p) + partials_bytes(p, n));
}

// Spill list of the tile engines (after the tile totals): [count][pad x3][tiles].
int32_t* spill_ptr(const Plan& p, void* ws, int64_t n) {
  return reinterpret_cast<int32_t*>(reinterpret_cast<uint8_t*>(tile_totals_ptr(p, ws, n)) +
                                    align_up(fory_amd::var_tile_totals_words(num_var_ops(p), n) * 8));
}

// Scan partials of the element string/binary columns (after the spill list): the
// element count is unknown when the workspace is sized, so their offsets are
// scanned in segments of kScanTile x (words - 1) elements (one segment in practice).
int64_t elem_partials_words(const Plan& p, int64_t n) {
  return p.generic || !elem_bytes_cols(p).empty() ? n / 8 + 8 : 0;
}

bool is_var_kind(int k) {
  return k == fory_amd::KIND_BYTES || k == fory_amd::KIND_LIST || k == fory_amd::KIND_MAP;
}

// Tree-engine launch: columns then the node table in the workspace. need_level:
// var columns of container depth <= need_level must carry offsets (encode: all of
// them; the decode values pass: all; decode_sizes checks levels itself).
int prepare_gen(const Plan& p, const fory_column* cols, int64_t n, int frame, void* ws, hipStream_t s,
                fory_amd::GenLaunch* L, int32_t need_level) {
  std::vector<ColumnDev> cd(p.nodes.size());
  for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
    const fory_amd::Node& nd = p.nodes[idx];
    const fory_column& c = cols[idx];
    if (n > 0 && is_var_kind(nd.kind) && p.gnodes[idx].cdepth <= need_level && !c.offsets)
      return fail(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(idx) + " needs offsets");
    if (n > 0 && need_level > 0 && p.gnodes[idx].cdepth == 0 && nd.kind != fory_amd::KIND_STRUCT &&
        !is_var_kind(nd.kind) && !c.values)  // (the sizes passes read no fixed values)
      return fail(FORY_ERR_INVALID_ARGUMENT, "column " + std::to_string(idx) + " has no values");
    ColumnDev d{};
    d.values = static_cast<const uint8_t*>(c.values);
    d.offsets = c.offsets;
    d.validity = nd.nullable ? c.validity : nullptr;
    d.out_values = static_cast<uint8_t*>(c.values);
    d.out_offsets = c.offsets;
    d.out_validity = nd.nullable ? c.validity : nullptr;
    cd[idx] = d;
  }
  const int64_t col_bytes = align_up((int64_t)cd.size() * (int64_t)sizeof(ColumnDev));
  std::vector<uint8_t> host((size_t)table_bytes(p), 0);
  std::memcpy(host.data(), cd.data(), cd.size() * sizeof(ColumnDev));
  std::memcpy(host.data() + col_bytes, p.gnodes.data(), p.gnodes.size() * sizeof(fory_amd::GNode));
  int rc = upload(ws, host.data(), (int64_t)host.size(), s);
  if (rc) return rc;
  L->cols = static_cast<const ColumnDev*>(ws);
  L->nodes = reinterpret_cast<const fory_amd::GNode*>(static_cast<uint8_t*>(ws) + col_bytes);
  L->num_nodes = (int32_t)p.gnodes.size();
  L->bitmap_bytes = p.bitmap_bytes;
  L->fixed_size = p.fixed_size;
  L->frame = frame;
  L->schema_hash = p.schema_hash;
  L->num_rows = n;
  L->fill_level = -1;
  L->max_depth = p.max_depth;
  return FORY_OK;
}

// --- columnar tree engine (treecol.hip) -------------------------------------
bool tc_var_kind(int k) { return k != fory_amd::KIND_FIXED && k != fory_amd::KIND_BOOL; }
bool tc_leaf_kind(int k) { return k == fory_amd::KIND_BYTES || k == fory_amd::KIND_DECIMAL; }
// Sizes (A): beans / lists / maps and item nodes; positions (P): beans / lists / maps.
bool tc_needs_sizes(const Plan& p, const fory_amd::TcVar& v) { return v.items || !tc_leaf_kind(p.nodes[v.node].kind); }
bool tc_needs_pos(const Plan& p, const fory_amd::TcVar& v) { return !tc_leaf_kind(p.nodes[v.node].kind); }
// Beans of leaf fields under a list / map: read by their container's items pass (decode).
// (Written inline by the encode's items pass they were not faster: measured 37.1 + 9.7 ms
// against 27.2 + 18.9 ms of tc_write_cont + tc_write_fields over the nested-shape bench,
// and the items kernel's extra registers slowed the lists of every plan.)
bool tc_inline_bean(const Plan& p, const fory_amd::TcVar& v) {
  return v.items && (p.gnodes[v.node].flags & fory_amd::kGNodeFlatBean);
}

void build_tc(fory_plan* plan) {
  const Plan& p = plan->p;
  TcInfo& t = plan->tc;
  const int N = (int)p.nodes.size();
  t.ok = p.generic && N > 0 && N <= fory_amd::kTcMaxNodes;
  if (!t.ok) return;
  t.parent.assign(N, -1);
  for (int i = 0; i < N; ++i)
    for (int32_t ch : p.nodes[i].children) t.parent[ch] = i;
  std::vector<int32_t> depth(N, 1);
  int maxd = 0;
  for (int i = 0; i < N; ++i) {  // pre-order: parents first
    depth[i] = t.parent[i] < 0 ? 1 : depth[t.parent[i]] + 1;
    if (tc_var_kind(p.nodes[i].kind)) maxd = std::max(maxd, depth[i]);
  }
  t.vidx.assign(N, -1);
  t.var.clear();
  for (int d = 1; d <= maxd; ++d) {  // var nodes by depth: parents are written before children
    for (int i = 0; i < N; ++i) {
      if (depth[i] != d || !tc_var_kind(p.nodes[i].kind)) continue;
      const int par = t.parent[i];
      fory_amd::TcVar v{};
      v.node = i;
      v.parent = par < 0 ? -1 : t.vidx[par];
      v.items = par >= 0 && p.nodes[par].kind != fory_amd::KIND_STRUCT;
      v.depth = d;
      t.vidx[i] = (int32_t)t.var.size();
      t.var.push_back(v);
    }
  }
}

// Instances of every node in this call: the rows at the top, a struct's children share
// its instances, items / keys / values are their column's length.
std::vector<int64_t> tc_domains(const fory_plan* plan, const fory_column* cols, int64_t n) {
  const TcInfo& t = plan->tc;
  const int N = (int)plan->p.nodes.size();
  std::vector<int64_t> m(N, 0);
  for (int i = 0; i < N; ++i) {
    const int par = t.parent[i];
    if (par < 0) m[i] = n;
    else if (plan->p.nodes[par].kind == fory_amd::KIND_STRUCT) m[i] = m[par];
    else m[i] = cols[i].length < 0 ? 0 : cols[i].length;
  }
  return m;
}

// Workspace after fory_rowfmt_workspace_bytes: the tables, item-scan partials, A arrays.
int64_t tc_bytes(const fory_plan* plan, const std::vector<int64_t>& m) {
  const TcInfo& t = plan->tc;
  int64_t maxm = 0, arrays = 0;
  for (const fory_amd::TcVar& v : t.var) {
    if (tc_needs_sizes(plan->p, v)) arrays += align_up((m[v.node] + 1) * 8);
    if (tc_needs_pos(plan->p, v)) arrays += align_up((m[v.node] + 1) * 8);
    if (v.items) maxm = std::max(maxm, m[v.node]);
  }
  const int64_t n = m.empty() ? 0 : m[0];  // (node 0 is top-level: the rows)
  return align_up((int64_t)sizeof(fory_amd::TcTables)) + align_up(fory_amd::tc_scan_flag_words(std::max(maxm, n)) * 8) +
         arrays;
}

bool tc_usable(const fory_plan* plan, const fory_column* cols, int64_t n, int64_t ws_bytes, int64_t* need) {
  if (!plan->tc.ok || !plan->p.kn.tree_col || n <= 0 || !cols) return false;
  const int64_t w = fory_rowfmt_workspace_bytes(plan, n) + tc_bytes(plan, tc_domains(plan, cols, n));
  if (need) *need = w;
  return ws_bytes >= w;
}

// Sizes of the last columnar encoded_size per workspace: encode reuses them when the
// plan, columns, rows and framing are the same and no other call used the workspace.
struct TcMemo {
  const void* ws = nullptr;
  uint64_t plan = 0, sig = 0;
};
std::mutex g_tc_mu;
TcMemo g_tc_memo[16];
int g_tc_next = 0;

uint64_t tc_signature(const fory_plan* plan, const fory_column* cols, int64_t n, int frame) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) {
    for (int b = 0; b < 8; ++b) h = (h ^ ((x >> (8 * b)) & 0xff)) * 1099511628211ull;
  };
  mix(plan->id);
  mix((uint64_t)n);
  mix((uint64_t)frame);
  for (size_t i = 0; i < plan->p.nodes.size(); ++i) {
    mix(reinterpret_cast<uintptr_t>(cols[i].values));
    mix(reinterpret_cast<uintptr_t>(cols[i].offsets));
    mix(reinterpret_cast<uintptr_t>(cols[i].validity));
    mix((uint64_t)cols[i].length);
  }
  return h;
}

void tc_forget(const void* ws) {
  if (!ws) return;
  std::lock_guard<std::mutex> lock(g_tc_mu);
  for (TcMemo& e : g_tc_memo)
    if (e.ws == ws) e = TcMemo{};
}

void tc_remember(const void* ws, uint64_t plan, uint64_t sig) {
  std::lock_guard<std::mutex> lock(g_tc_mu);
  TcMemo* slot = nullptr;
  for (TcMemo& e : g_tc_memo)
    if (e.ws == ws) slot = &e;
  if (!slot) slot = &g_tc_memo[g_tc_next++ & 15];
  *slot = TcMemo{ws, plan, sig};
}

bool tc_recall(const void* ws, uint64_t plan, uint64_t sig) {
  std::lock_guard<std::mutex> lock(g_tc_mu);
  for (const TcMemo& e : g_tc_memo)
    if (e.ws == ws && e.plan == plan && e.sig == sig) return true;
  return false;
}

// Tables of a columnar call into the workspace (after the per-lane engine's region).
int tc_prepare(const fory_plan* plan, const fory_column* cols, int64_t n, void* ws, hipStream_t s,
               fory_amd::TcTables* T, const fory_amd::TcTables** dT, int64_t** partials) {
  const TcInfo& t = plan->tc;
  const std::vector<int64_t> m = tc_domains(plan, cols, n);
  uint8_t* base = static_cast<uint8_t*>(ws) + fory_rowfmt_workspace_bytes(plan, n);
  std::memset(T, 0, sizeof(*T));
  int64_t maxm = 0;
  for (const fory_amd::TcVar& v : t.var)
    if (v.items) maxm = std::max(maxm, m[v.node]);
  uint8_t* at = base + align_up((int64_t)sizeof(fory_amd::TcTables));
  *partials = reinterpret_cast<int64_t*>(at);  // look-back flags of the fused size scans
  at += align_up(fory_amd::tc_scan_flag_words(std::max(maxm, n)) * 8);
  for (size_t i = 0; i < m.size(); ++i) {
    T->m[i] = m[i];
    T->vidx[i] = t.vidx[i];
  }
  for (size_t v = 0; v < t.var.size(); ++v) {
    T->var[v] = t.var[v];
    const int node = t.var[v].node;
    if (tc_needs_sizes(plan->p, t.var[v])) {
      T->A[node] = reinterpret_cast<int64_t*>(at);
      at += align_up((m[node] + 1) * 8);
    }
    if (tc_needs_pos(plan->p, t.var[v])) {
      T->P[node] = reinterpret_cast<int64_t*>(at);
      at += align_up((m[node] + 1) * 8);
    }
  }
  T->nvar = (int32_t)t.var.size();
  T->depths = t.var.empty() ? 0 : t.var.back().depth;
  int nk = 0;  // fields by parent: the rows', then each bean's
  for (int32_t f : plan->p.top) T->kids[nk++] = f;
  T->nroot = nk;
  for (size_t i = 0; i < plan->p.nodes.size(); ++i) {
    if (plan->p.nodes[i].kind != fory_amd::KIND_STRUCT) continue;
    T->kid0[i] = nk;
    for (int32_t ch : plan->p.nodes[i].children) T->kids[nk++] = ch;
  }
  *dT = reinterpret_cast<const fory_amd::TcTables*>(base);
  return upload(base, T, (int64_t)sizeof(*T), s);
}

// Bottom-up sizes of every var node (children before parents), item nodes scanned.
int tc_sizes(const fory_plan* plan, const fory_amd::GenLaunch& G, const fory_amd::TcTables& T,
             const fory_amd::TcTables* dT, int64_t* partials, hipStream_t s) {
  const TcInfo& t = plan->tc;
  for (int v = (int)t.var.size() - 1; v >= 0; --v) {  // deepest first
    const fory_amd::TcVar& tv = t.var[(size_t)v];
    if (!tc_needs_sizes(plan->p, tv)) continue;  // strings / decimals in rows and beans: sized in place
    const int64_t m = T.m[tv.node];
    const bool root_coll = G.frame == FORY_FRAME_COLLECTION && tv.node == 0;
    const hipError_t e = tv.items ? fory_amd::launch_tc_size_scan(G, dT, tv.node, m, root_coll, T.A[tv.node],
                                                                  reinterpret_cast<uint64_t*>(partials), s)
                                  : fory_amd::launch_tc_sizes(G, dT, tv.node, m, root_coll, s);
    if (e != hipSuccess) return hip_fail(e, "tc_sizes");
  }
  return FORY_OK;
}

// --- columnar decode (treedec.hip) ------------------------------------------------
// Positions (P, SZ, TL) of the bean / list / map instances known in this call.
// (then the scan partials of a level's Arrow offsets columns, scanned together)
int64_t td_partials_words(const fory_plan* plan, const std::vector<int64_t>& m) {
  int64_t w = 0;
  for (size_t i = 0; i < plan->p.nodes.size(); ++i)
    if (is_var_kind(plan->p.nodes[i].kind)) w += fory_amd::scan_batch_partials(m[i]);
  return w;
}

int64_t td_bytes(const fory_plan* plan, const std::vector<int64_t>& m) {
  int64_t b = align_up((int64_t)sizeof(fory_amd::TdTables));
  for (const fory_amd::TcVar& v : plan->tc.var) {
    if (tc_needs_pos(plan->p, v)) b += align_up((m[v.node] + 1) * 8) + 2 * align_up((m[v.node] + 1) * 4);
    if (plan->p.nodes[v.node].kind == fory_amd::KIND_BYTES) b += align_up((m[v.node] + 1) * 8);
  }
  return b + align_up(td_partials_words(plan, m) * 8);
}

bool td_usable(const fory_plan* plan, const fory_column* out_cols, int64_t n, int64_t ws_bytes) {
  if (!plan->tc.ok || !plan->p.kn.tree_col || n <= 0 || !out_cols) return false;
  return ws_bytes >= fory_rowfmt_workspace_bytes(plan, n) + td_bytes(plan, tc_domains(plan, out_cols, n));
}

int td_prepare(const fory_plan* plan, const fory_column* out_cols, int64_t n, void* ws, hipStream_t s,
               const fory_amd::TdTables** dT, std::vector<int64_t>* m, int64_t** partials = nullptr,
               fory_amd::TdTables* host = nullptr) {
  *m = tc_domains(plan, out_cols, n);
  uint8_t* base = static_cast<uint8_t*>(ws) + fory_rowfmt_workspace_bytes(plan, n);
  fory_amd::TdTables T;
  std::memset(&T, 0, sizeof(T));
  uint8_t* at = base + align_up((int64_t)sizeof(fory_amd::TdTables));
  // by decode level: a level's arrays stay where they are when deeper levels are allocated
  // (string sources with their level: td_strings copies them in the decode call)
  for (int32_t cd = 0; cd <= plan->p.max_cdepth; ++cd)
    for (const fory_amd::TcVar& v : plan->tc.var) {
      if (plan->p.gnodes[v.node].cdepth != cd) continue;
      const int64_t k = (*m)[v.node] + 1;
      if (plan->p.nodes[v.node].kind == fory_amd::KIND_BYTES) {
        T.SRC[v.node] = reinterpret_cast<int64_t*>(at);
        at += align_up(k * 8);
      }
      if (!tc_needs_pos(plan->p, v)) continue;
      T.P[v.node] = reinterpret_cast<int64_t*>(at);
      at += align_up(k * 8);
      T.SZ[v.node] = reinterpret_cast<int32_t*>(at);
      at += align_up(k * 4);
      T.TL[v.node] = reinterpret_cast<int32_t*>(at);
      at += align_up(k * 4);
    }
  if (partials) *partials = reinterpret_cast<int64_t*>(at);
  for (size_t i = 0; i < m->size(); ++i) T.m[i] = (*m)[i];
  int nk = 0;
  for (int32_t f : plan->p.top) T.kids[nk++] = f;
  T.nroot = nk;
  for (size_t i = 0; i < plan->p.nodes.size(); ++i) {
    if (plan->p.nodes[i].kind != fory_amd::KIND_STRUCT) continue;
    T.kid0[i] = nk;
    for (int32_t ch : plan->p.nodes[i].children) T.kids[nk++] = ch;
  }
  *dT = reinterpret_cast<const fory_amd::TdTables*>(base);
  if (host) *host = T;
  return upload(base, &T, (int64_t)sizeof(T), s);
}

// Levels the last columnar decode_sizes on a workspace ran: the next call with the same
// plan, rows, row offsets and the same columns down to that level resumes after it
// (the Python mirror and a JNI caller size one level per call).
struct TdMemo {
  const void* ws = nullptr;
  uint64_t plan = 0, sig = 0;
  int32_t level = -1;
};
std::mutex g_td_mu;
TdMemo g_td_memo[16];
int g_td_next = 0;

uint64_t td_signature(const fory_plan* plan, const void* rows, const int64_t* offs, int64_t n, int frame,
                      const fory_column* cols, int32_t level) {
  uint64_t h = 1469598103934665603ull;
  auto mix = [&](uint64_t x) {
    for (int b = 0; b < 8; ++b) h = (h ^ ((x >> (8 * b)) & 0xff)) * 1099511628211ull;
  };
  mix(plan->id);
  mix(reinterpret_cast<uintptr_t>(rows));
  mix(reinterpret_cast<uintptr_t>(offs));
  mix((uint64_t)n);
  mix((uint64_t)frame);
  mix((uint64_t)(int64_t)level);
  for (size_t i = 0; i < plan->p.nodes.size(); ++i) {
    if (plan->p.gnodes[i].cdepth > level) continue;
    // string / binary bytes are allocated after their level is sized: not an input here
    if (plan->p.nodes[i].kind != fory_amd::KIND_BYTES) mix(reinterpret_cast<uintptr_t>(cols[i].values));
    mix(reinterpret_cast<uintptr_t>(cols[i].offsets));
    mix(reinterpret_cast<uintptr_t>(cols[i].validity));
    mix((uint64_t)cols[i].length);
  }
  return h;
}

void td_forget(const void* ws) {
  if (!ws) return;
  std::lock_guard<std::mutex> lock(g_td_mu);
  for (TdMemo& e : g_td_memo)
    if (e.ws == ws) e = TdMemo{};
}

void td_remember(const fory_plan* plan, const void* ws, const void* rows, const int64_t* offs, int64_t n, int frame,
                 const fory_column* cols, int32_t level) {
  td_forget(ws);
  if (level < 0) return;
  const uint64_t sig = td_signature(plan, rows, offs, n, frame, cols, level);
  std::lock_guard<std::mutex> lock(g_td_mu);
  g_td_memo[g_td_next++ & 15] = TdMemo{ws, plan->id, sig, level};
}

// The last level done on this workspace for these inputs, or -1.
int32_t td_recall(const fory_plan* plan, const void* ws, const void* rows, const int64_t* offs, int64_t n, int frame,
                  const fory_column* cols) {
  TdMemo e;
  {
    std::lock_guard<std::mutex> lock(g_td_mu);
    for (const TdMemo& x : g_td_memo)
      if (x.ws == ws && x.plan == plan->id) e = x;
  }
  if (!e.ws || td_signature(plan, rows, offs, n, frame, cols, e.level) != e.sig) return -1;
  return e.level;
}

// The passes of one decode level, parents first. level >= 0: its counts (and the
// positions of its beans / lists / maps) from the rows (level 0), the items of the
// level-(L-1) lists / maps and the level-L beans, given the positions the passes of the
// levels before it left in the workspace in this call; -1: every value, every pass.
int td_run(const fory_plan* plan, fory_amd::GenLaunch G, const fory_amd::TdTables* dT, const std::vector<int64_t>& m,
           int level, const void* rows, const int64_t* offs, int32_t* status, hipStream_t s) {
  const Plan& p = plan->p;
  G.fill_level = level;
  const uint8_t* r = static_cast<const uint8_t*>(rows);
  hipError_t e = hipSuccess;
  if (level <= 0) e = fory_amd::launch_td_rows(G, dT, (int)p.top.size(), r, offs, status, s);
  for (size_t v = 0; v < plan->tc.var.size() && e == hipSuccess; ++v) {
    const int node = plan->tc.var[v].node;
    const int kind = p.nodes[node].kind;
    const int cd = p.gnodes[node].cdepth;
    if (!tc_needs_pos(p, plan->tc.var[v]) || tc_inline_bean(p, plan->tc.var[v])) continue;
    if (level >= 0 && (kind == fory_amd::KIND_STRUCT ? cd != level : cd != level - 1)) continue;
    int iflags = 0;  // the item nodes' flags (a list's item, a map's key and value)
    if (kind == fory_amd::KIND_LIST || kind == fory_amd::KIND_MAP) {
      iflags = p.gnodes[node + 1].flags;
      if (kind == fory_amd::KIND_MAP) iflags |= p.gnodes[p.gnodes[node + 1].end].flags;
    }
    e = fory_amd::launch_td_node(G, dT, node, m[node], kind, (int)p.nodes[node].children.size(), iflags, r, status, s);
  }
  return e == hipSuccess ? FORY_OK : hip_fail(e, "td_decode");
}

int64_t* elem_partials_ptr(const Plan& p, void* ws, int64_t n) {
  return reinterpret_cast<int64_t*>(reinterpret_cast<uint8_t*>(spill_ptr(p, ws, n)) +
                                    align_up(fory_amd::var_spill_words(n) * 4));
}

}  // namespace

extern "C" {

int32_t fory_rowfmt_abi_version(void) { return FORY_ROWFMT_ABI_VERSION; }

// Debug only (not in the public header): copies the flat-kernel phase timeline
// recorded under FORY_ROWFMT_VARPROF=1 (8 s_memrealtime stamps per tile).
int64_t fory_rowfmt_debug_timeline(uint64_t* host, int64_t max_words) {
  return fory_amd::var_prof_copy(host, max_words);
}

const char* fory_rowfmt_last_error(void) { return g_err.c_str(); }

// Library-internal (host.cpp): a stream about to be destroyed (its work complete) —
// slots whose last copy was queued on it are waited for now, while the stream is
// alive, and never queried again through an event of a destroyed stream.
void fory_rowfmt_internal_retire_stream(void* stream) {
  std::vector<UploadRing*> rings;
  {
    std::lock_guard<std::mutex> lock(g_rings_mu);
    for (auto& kv : *g_rings) rings.push_back(kv.second);
  }
  for (UploadRing* r : rings) {
    std::lock_guard<std::mutex> lock(r->mu);
    for (UploadSlot* sl : r->slots)
      if (sl->pending && !sl->busy && sl->st == static_cast<hipStream_t>(stream)) {
        (void)hipEventSynchronize(sl->ev);
        sl->pending = false;
      }
  }
}

// Library-internal (host.cpp): shares last_error and the planner's column layout.
int fory_rowfmt_internal_set_error(int code, const char* msg) { return fail(code, msg); }

int fory_rowfmt_internal_column_layout(const fory_plan* plan, int32_t* width, int32_t* nullable) {
  const Plan& p = plan->p;
  for (size_t i = 0; i < p.nodes.size(); ++i) {
    width[i] = p.nodes[i].width;
    nullable[i] = p.nodes[i].nullable;
  }
  return FORY_OK;
}

// kind (FieldKind), width, nullable and parent node (-1: top level) of every pre-order node.
int fory_rowfmt_internal_node_layout(const fory_plan* plan, int32_t* kind, int32_t* width, int32_t* nullable,
                                     int32_t* parent) {
  const Plan& p = plan->p;
  for (size_t i = 0; i < p.nodes.size(); ++i) {
    kind[i] = p.nodes[i].kind;
    width[i] = p.nodes[i].width;
    if (kind[i] == fory_amd::KIND_DECIMAL) kind[i] = fory_amd::KIND_FIXED, width[i] = 16;  // a 16-byte column
    nullable[i] = p.nodes[i].nullable;
    parent[i] = -1;
  }
  for (size_t i = 0; i < p.nodes.size(); ++i)
    for (int32_t ch : p.nodes[i].children) parent[ch] = (int32_t)i;
  return FORY_OK;
}

int fory_rowfmt_plan_create(const fory_field_desc* fields, int32_t num_desc, fory_plan** out_plan) {
  if (!out_plan) return fail(FORY_ERR_INVALID_ARGUMENT, "out_plan is null");
  *out_plan = nullptr;
  fory_plan* plan = new fory_plan();
  std::string err;
  int rc = fory_amd::build_plan(fields, num_desc, &plan->p, &err);
  if (rc) {
    delete plan;
    return fail(rc, "Create encoder failed: " + err);
  }
  if (!plan->p.fixed_width && !plan->p.generic && plan->p.max_depth > 8) {
    delete plan;
    return fail(FORY_ERR_UNSUPPORTED, "device path supports struct nesting depth <= 8");
  }
  plan->p.kn = fory_amd::knobs_from_env();  // launch knobs fixed for the plan's life
  build_tc(plan);
  static std::atomic<uint64_t> next_id{1};
  plan->id = next_id++;
  *out_plan = plan;
  return FORY_OK;
}

void fory_rowfmt_plan_destroy(fory_plan* plan) { delete plan; }

int fory_rowfmt_plan_info(const fory_plan* plan, fory_plan_info* info) {
  if (!plan || !info) return fail(FORY_ERR_INVALID_ARGUMENT, "plan or info is null");
  const Plan& p = plan->p;
  info->schema_hash = p.schema_hash;
  info->num_fields = (int32_t)p.top.size();
  info->num_columns = (int32_t)p.nodes.size();
  info->bitmap_bytes = p.bitmap_bytes;
  info->fixed_size = p.fixed_size;
  info->fixed_width = p.fixed_width ? 1 : 0;
  info->row_size = p.fixed_width ? p.fixed_size : -1;
  return FORY_OK;
}

int64_t fory_rowfmt_workspace_bytes(const fory_plan* plan, int64_t num_rows) {
  if (!plan) return -1;
  const int64_t n = num_rows < 0 ? 0 : num_rows;
  return table_bytes(plan->p) + partials_bytes(plan->p, n) +
         align_up(fory_amd::var_tile_totals_words(num_var_ops(plan->p), n) * 8) +
         align_up(fory_amd::var_spill_words(n) * 4) + align_up(elem_partials_words(plan->p, n) * 8);
}

int64_t fory_rowfmt_encode_workspace_bytes(const fory_plan* plan, const fory_column* cols, int64_t num_rows) {
  if (!plan) return -1;
  const int64_t base = fory_rowfmt_workspace_bytes(plan, num_rows);
  if (!plan->tc.ok || !plan->p.kn.tree_col || num_rows <= 0 || !cols) return base;
  return base + tc_bytes(plan, tc_domains(plan, cols, num_rows));
}

int64_t fory_rowfmt_decode_workspace_bytes(const fory_plan* plan, const fory_column* out_cols, int64_t num_rows) {
  if (!plan) return -1;
  const int64_t base = fory_rowfmt_workspace_bytes(plan, num_rows);
  if (!plan->tc.ok || !plan->p.kn.tree_col || num_rows <= 0 || !out_cols) return base;
  return base + td_bytes(plan, tc_domains(plan, out_cols, num_rows));
}

int fory_rowfmt_encoded_size(const fory_plan* plan, const fory_column* cols, int64_t num_rows,
                             int32_t frame_mode, int64_t* d_row_offsets, void* d_workspace,
                             int64_t workspace_bytes, void* stream) {
  int rc = check_common(plan, cols, num_rows, frame_mode, d_workspace, workspace_bytes);
  if (rc) return rc;
  if (!d_row_offsets) return fail(FORY_ERR_INVALID_ARGUMENT, "d_row_offsets is null");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Plan& p = plan->p;
  hipError_t e;
  if (p.fixed_width) {
    e = fory_amd::launch_fill_offsets(d_row_offsets, num_rows, p.fixed_size + fory_amd::frame_header_bytes(frame_mode), s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "fill_offsets");
  }
  if (num_rows == 0) {
    e = hipMemsetAsync(d_row_offsets, 0, sizeof(int64_t), s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "hipMemsetAsync");
  }
  if (p.generic) {
    fory_amd::GenLaunch G{};
    rc = prepare_gen(p, cols, num_rows, frame_mode, d_workspace, s, &G, 1 << 20);
    if (rc) return rc;
    if (tc_usable(plan, cols, num_rows, workspace_bytes, nullptr)) {  // columnar: node sizes, then the rows
      fory_amd::TcTables T;
      const fory_amd::TcTables* dT = nullptr;
      int64_t* tpart = nullptr;
      rc = tc_prepare(plan, cols, num_rows, d_workspace, s, &T, &dT, &tpart);
      if (!rc) rc = tc_sizes(plan, G, T, dT, tpart, s);
      if (rc) return rc;
      e = fory_amd::launch_tc_size_scan(G, dT, -1, num_rows, false, d_row_offsets, reinterpret_cast<uint64_t*>(tpart), s);
      if (e != hipSuccess) return hip_fail(e, "tc_rows");
      tc_remember(d_workspace, plan->id, tc_signature(plan, cols, num_rows, frame_mode));
      return FORY_OK;
    }
    e = fory_amd::launch_gen_sizes(G, d_row_offsets, s);
    if (e != hipSuccess) return hip_fail(e, "gen_sizes");
    e = fory_amd::launch_scan_i64(d_row_offsets, num_rows, partials_ptr(p, d_workspace), s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "scan");
  }
  fory_amd::VarLaunch L{};
  rc = prepare_var(p, cols, num_rows, frame_mode, d_workspace, s, &L);
  if (rc) return rc;
  e = fory_amd::launch_var_sizes(L, d_row_offsets, s);
  if (e != hipSuccess) return hip_fail(e, "var_sizes");
  e = fory_amd::launch_scan_i64(d_row_offsets, num_rows, partials_ptr(p, d_workspace), s);
  return e == hipSuccess ? FORY_OK : hip_fail(e, "scan");
}

int fory_rowfmt_encode(const fory_plan* plan, const fory_column* cols, int64_t num_rows,
                       int32_t frame_mode, const int64_t* d_row_offsets, void* d_out,
                       int64_t out_capacity, int32_t* d_status, void* d_workspace,
                       int64_t workspace_bytes, void* stream) {
  int rc = check_common(plan, cols, num_rows, frame_mode, d_workspace, workspace_bytes, KEEP_TC);
  if (rc) return rc;
  if (!plan->p.generic || !tc_usable(plan, cols, num_rows, workspace_bytes, nullptr)) tc_forget(d_workspace);
  if (num_rows == 0) return FORY_OK;
  if (!d_out) return fail(FORY_ERR_INVALID_ARGUMENT, "d_out is null");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Plan& p = plan->p;
  hipError_t e;
  if (use_tiled(p, frame_mode)) {
    const int64_t stride = p.fixed_size + fory_amd::frame_header_bytes(frame_mode);
    if (num_rows * stride > out_capacity)
      return fail(FORY_ERR_CAPACITY, "output capacity " + std::to_string(out_capacity) + " < " +
                                         std::to_string(num_rows * stride) + " bytes");
    if (reinterpret_cast<uintptr_t>(d_out) & 15)
      return fail(FORY_ERR_INVALID_ARGUMENT, "d_out must be 16-byte aligned");
    std::vector<FixedFieldDev> tab;
    rc = bind_fixed(p, cols, num_rows, false, &tab);
    if (rc) return rc;
    fory_amd::FixedLaunch L = fixed_launch(p, d_workspace, num_rows, frame_mode);
    rc = upload_fixed_tables(p, d_workspace, tab, false, s, &L.valid8);
    if (rc) return rc;
    e = fory_amd::launch_encode_fixed(L, static_cast<uint8_t*>(d_out), s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "encode_fixed");
  }
  if (p.fixed_width)
    return fail(FORY_ERR_UNSUPPORTED, "row too wide for the device path");
  if (!d_row_offsets)
    return fail(FORY_ERR_INVALID_ARGUMENT, "varlen schema: d_row_offsets (from encoded_size) required");
  if (p.generic) {
    fory_amd::GenLaunch G{};
    rc = prepare_gen(p, cols, num_rows, frame_mode, d_workspace, s, &G, 1 << 20);
    if (rc) return rc;
    if (tc_usable(plan, cols, num_rows, workspace_bytes, nullptr) && !(reinterpret_cast<uintptr_t>(d_out) & 3)) {
      fory_amd::TcTables T;
      const fory_amd::TcTables* dT = nullptr;
      int64_t* tpart = nullptr;
      const uint64_t sig = tc_signature(plan, cols, num_rows, frame_mode);
      rc = tc_prepare(plan, cols, num_rows, d_workspace, s, &T, &dT, &tpart);
      // sizes the preceding encoded_size left for these columns are used once: encode
      // never leaves sizes of its own, so a later encode of refilled columns re-sizes them
      const bool left = !rc && tc_recall(d_workspace, plan->id, sig);
      tc_forget(d_workspace);
      if (!rc && !left) rc = tc_sizes(plan, G, T, dT, tpart, s);
      if (rc) return rc;
      uint8_t* out = static_cast<uint8_t*>(d_out);
      e = fory_amd::launch_tc_write_rows(G, dT, T.nroot, d_row_offsets, out, out_capacity, d_status, s);
      for (size_t v = 0; v < plan->tc.var.size() && e == hipSuccess; ++v) {
        const int node = plan->tc.var[v].node;
        if (!tc_needs_pos(p, plan->tc.var[v])) continue;  // written by their parents
        const int key = node + 1;  // a list's items / a map's keys, then its values (pre-order)
        const bool cont = p.gnodes[node].kind == fory_amd::KIND_LIST || p.gnodes[node].kind == fory_amd::KIND_MAP;
        const int kk = cont ? p.gnodes[key].kind : 0;
        const int vk = p.gnodes[node].kind == fory_amd::KIND_MAP ? p.gnodes[p.gnodes[key].end].kind : 0;
        e = fory_amd::launch_tc_write_node(G, dT, node, T.m[node], out, out_capacity, d_status, s, p.nodes[node].kind,
                                           (int)p.nodes[node].children.size(), kk, vk);
      }
      return e == hipSuccess ? FORY_OK : hip_fail(e, "tc_write");
    }
    e = fory_amd::launch_gen_encode(G, d_row_offsets, static_cast<uint8_t*>(d_out), out_capacity, d_status, s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "gen_encode");
  }
  fory_amd::VarLaunch L{};
  rc = prepare_var(p, cols, num_rows, frame_mode, d_workspace, s, &L);
  if (rc) return rc;
  e = fory_amd::launch_var_encode(L, d_row_offsets, static_cast<uint8_t*>(d_out), out_capacity, d_status, s);
  return e == hipSuccess ? FORY_OK : hip_fail(e, "var_encode");
}

int fory_rowfmt_decode_sizes(const fory_plan* plan, const void* d_rows, const int64_t* d_row_offsets,
                             int64_t num_rows, int32_t frame_mode, const fory_column* out_cols,
                             int32_t* d_status, void* d_workspace, int64_t workspace_bytes,
                             void* stream) {
  int rc = check_common(plan, out_cols, num_rows, frame_mode, d_workspace, workspace_bytes, KEEP_TD);
  if (rc) return rc;
  const Plan& p = plan->p;
  if (p.fixed_width || num_rows == 0) {
    if (!p.fixed_width) {
      hipStream_t s0 = static_cast<hipStream_t>(stream);
      for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
        const int k = p.nodes[idx].kind;
        if ((k == fory_amd::KIND_BYTES || k == fory_amd::KIND_LIST || k == fory_amd::KIND_MAP) && out_cols &&
            out_cols[idx].offsets)
          (void)hipMemsetAsync(out_cols[idx].offsets, 0, sizeof(int32_t), s0);
      }
    }
    return FORY_OK;
  }
  if (!d_rows || !d_row_offsets)
    return fail(FORY_ERR_INVALID_ARGUMENT, "varlen schema: d_rows and d_row_offsets required");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (p.generic) {
    // Container depth 0 (the rows' own strings / lists / maps), then each deeper depth
    // whose columns the caller has allocated (positions = the totals of the level above).
    fory_amd::GenLaunch G{};
    rc = prepare_gen(p, out_cols, num_rows, frame_mode, d_workspace, s, &G, 0);
    if (rc) return rc;
    const bool columnar = td_usable(plan, out_cols, num_rows, workspace_bytes);
    const fory_amd::TdTables* dT = nullptr;
    fory_amd::TdTables Th{};
    std::vector<int64_t> m;
    int64_t* td_part = nullptr;
    // columnar: the levels run in order, each from the positions the one before left; the
    // levels the previous call on this workspace ran (same plan, rows and columns) are done
    int32_t first = 0, last = -1;
    if (columnar) {
      rc = td_prepare(plan, out_cols, num_rows, d_workspace, s, &dT, &m, &td_part, &Th);
      if (rc) return rc;
      first = td_recall(plan, d_workspace, d_rows, d_row_offsets, num_rows, frame_mode, out_cols) + 1;
      last = first - 1;
    } else {
      td_forget(d_workspace);
    }
    for (int32_t level = 0; level <= p.max_cdepth; ++level) {
      bool any = false, ready = true;
      for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
        if (!is_var_kind(p.nodes[idx].kind) || p.gnodes[idx].cdepth != level) continue;
        any = true;
        if (!out_cols[idx].offsets || out_cols[idx].length < 0) ready = false;
      }
      if (!any || !ready) break;
      if (level < first) continue;  // counts and positions left by the previous call
      hipError_t e = hipSuccess;
      if (columnar) {  // columnar: this level's passes
        for (size_t idx = 0; idx < p.nodes.size(); ++idx)  // string sources: -1 until a pass records one
          if (p.nodes[idx].kind == fory_amd::KIND_BYTES && p.gnodes[idx].cdepth == level && Th.SRC[idx]) {
            e = hipMemsetAsync(Th.SRC[idx], 0xff, (size_t)(m[idx] + 1) * 8, s);
            if (e != hipSuccess) return hip_fail(e, "hipMemsetAsync");
          }
        rc = td_run(plan, G, dT, m, level, d_rows, d_row_offsets, d_status, s);
        if (rc) return rc;
        last = level;
      } else {
        G.fill_level = level;
        e = fory_amd::launch_gen_decode(G, static_cast<const uint8_t*>(d_rows), d_row_offsets, d_status, s);
        if (e != hipSuccess) return hip_fail(e, "gen_decode (lengths)");
      }
      if (columnar) {  // the level's offsets columns in one set of launches
        std::vector<int32_t*> cs;
        std::vector<int64_t> ns;
        for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
          if (!is_var_kind(p.nodes[idx].kind) || p.gnodes[idx].cdepth != level) continue;
          cs.push_back(out_cols[idx].offsets);
          ns.push_back(m[idx]);  // the instances of the column (the workspace's partials are sized by them)
        }
        e = fory_amd::launch_scan_offsets_batch(cs.data(), ns.data(), (int)cs.size(), td_part, d_status, s);
        if (e != hipSuccess) return hip_fail(e, "scan offsets");
        continue;
      }
      for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
        if (!is_var_kind(p.nodes[idx].kind) || p.gnodes[idx].cdepth != level) continue;
        e = level == 0 ? fory_amd::launch_scan_offsets_i32(out_cols[idx].offsets, num_rows,
                                                           partials_ptr(p, d_workspace), d_status, s)
                       : fory_amd::launch_scan_offsets_i32_segmented(
                             out_cols[idx].offsets, out_cols[idx].length, elem_partials_ptr(p, d_workspace, num_rows),
                             elem_partials_words(p, num_rows), d_status, s);
        if (e != hipSuccess) return hip_fail(e, "scan offsets");
      }
    }
    if (columnar) td_remember(plan, d_workspace, d_rows, d_row_offsets, num_rows, frame_mode, out_cols, last);
    return FORY_OK;
  }
  fory_amd::VarLaunch L{};
  rc = prepare_var(p, out_cols, num_rows, frame_mode, d_workspace, s, &L, true);
  if (rc) return rc;
  hipError_t e = fory_amd::launch_var_decode_lengths(L, static_cast<const uint8_t*>(d_rows), d_row_offsets,
                                                     tile_totals_ptr(p, d_workspace, num_rows),
                                                     partials_ptr(p, d_workspace), d_status, s);
  if (e != hipSuccess) return hip_fail(e, "var_decode_lengths");
  if (fory_amd::var_decode_tiled_offsets(L)) return FORY_OK;  // tile bases written; decode fills the rest
  const std::vector<int32_t> elem = elem_bytes_cols(p);
  auto is_elem = [&](size_t idx) { return std::find(elem.begin(), elem.end(), (int32_t)idx) != elem.end(); };
  for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
    const int k = p.nodes[idx].kind;
    if (k != fory_amd::KIND_BYTES && k != fory_amd::KIND_LIST && k != fory_amd::KIND_MAP) continue;
    if (is_elem(idx)) continue;
    e = fory_amd::launch_scan_offsets_i32(out_cols[idx].offsets, num_rows, partials_ptr(p, d_workspace),
                                          d_status, s);
    if (e != hipSuccess) return hip_fail(e, "scan offsets");
  }
  // pass 2: element string/binary columns whose offsets the caller has allocated
  // (length = the container's element total from pass 1)
  bool level2 = false;
  for (int32_t idx : elem) {
    if (!out_cols[idx].offsets) continue;
    if (out_cols[idx].length < 0) return fail(FORY_ERR_INVALID_ARGUMENT, "element column length < 0");
    level2 = true;
  }
  if (!level2) return FORY_OK;
  L.level2 = 1;
  e = fory_amd::launch_var_decode_lengths(L, static_cast<const uint8_t*>(d_rows), d_row_offsets,
                                          tile_totals_ptr(p, d_workspace, num_rows), partials_ptr(p, d_workspace),
                                          d_status, s);
  if (e != hipSuccess) return hip_fail(e, "var_decode_lengths (elements)");
  for (int32_t idx : elem) {
    if (!out_cols[idx].offsets) continue;
    e = fory_amd::launch_scan_offsets_i32_segmented(out_cols[idx].offsets, out_cols[idx].length,
                                                    elem_partials_ptr(p, d_workspace, num_rows),
                                                    elem_partials_words(p, num_rows), d_status, s);
    if (e != hipSuccess) return hip_fail(e, "scan element offsets");
  }
  return FORY_OK;
}

int fory_rowfmt_decode(const fory_plan* plan, const void* d_rows, const int64_t* d_row_offsets,
                       int64_t num_rows, int32_t frame_mode, const fory_column* out_cols,
                       int32_t* d_status, void* d_workspace, int64_t workspace_bytes, void* stream) {
  int rc = check_common(plan, out_cols, num_rows, frame_mode, d_workspace, workspace_bytes, KEEP_TD);
  if (rc || !plan->p.generic || !td_usable(plan, out_cols, num_rows, workspace_bytes)) td_forget(d_workspace);
  if (rc) return rc;
  if (num_rows == 0) return FORY_OK;
  if (!d_rows) return fail(FORY_ERR_INVALID_ARGUMENT, "d_rows is null");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Plan& p = plan->p;
  hipError_t e;
  if (use_tiled(p, frame_mode)) {
    if (reinterpret_cast<uintptr_t>(d_rows) & 15)
      return fail(FORY_ERR_INVALID_ARGUMENT, "d_rows must be 16-byte aligned");
    std::vector<FixedFieldDev> tab;
    rc = bind_fixed(p, out_cols, num_rows, true, &tab);
    if (rc) return rc;
    fory_amd::FixedLaunch L = fixed_launch(p, d_workspace, num_rows, frame_mode);
    rc = upload_fixed_tables(p, d_workspace, tab, true, s, &L.valid8);
    if (rc) return rc;
    L.cols_aligned16 = 1;
    for (const FixedFieldDev& f : tab)
      if (reinterpret_cast<uintptr_t>(f.out_values) & 15) L.cols_aligned16 = 0;
    e = fory_amd::launch_decode_fixed(L, static_cast<const uint8_t*>(d_rows), d_status, s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "decode_fixed");
  }
  if (p.fixed_width) return fail(FORY_ERR_UNSUPPORTED, "row too wide for the device path");
  if (!d_row_offsets)
    return fail(FORY_ERR_INVALID_ARGUMENT, "varlen schema: d_row_offsets required");
  if (p.generic) {
    fory_amd::GenLaunch G{};
    rc = prepare_gen(p, out_cols, num_rows, frame_mode, d_workspace, s, &G, 1 << 20);
    if (rc) return rc;
    if (td_usable(plan, out_cols, num_rows, workspace_bytes)) {  // columnar
      const fory_amd::TdTables* dT = nullptr;
      fory_amd::TdTables Th;
      std::vector<int64_t> m;
      rc = td_prepare(plan, out_cols, num_rows, d_workspace, s, &dT, &m, nullptr, &Th);
      if (rc) return rc;
      // decode_sizes on this workspace ran every level with var columns: their passes
      // wrote all but the string bytes. Run the levels below them (fixed-width items
      // only), then copy the bytes from the recorded positions. Else every node's values.
      const int32_t done = td_recall(plan, d_workspace, d_rows, d_row_offsets, num_rows, frame_mode, out_cols);
      td_forget(d_workspace);
      bool rest_fixed = done >= 0;
      for (size_t idx = 0; idx < p.nodes.size() && rest_fixed; ++idx)
        if (is_var_kind(p.nodes[idx].kind) && p.gnodes[idx].cdepth > done) rest_fixed = false;
      if (!rest_fixed) return td_run(plan, G, dT, m, -1, d_rows, d_row_offsets, d_status, s);
      for (int32_t level = done + 1; level <= p.max_cdepth; ++level) {
        rc = td_run(plan, G, dT, m, level, d_rows, d_row_offsets, d_status, s);
        if (rc) return rc;
      }
      for (size_t idx = 0; idx < p.nodes.size(); ++idx) {
        if (p.nodes[idx].kind != fory_amd::KIND_BYTES) continue;
        e = fory_amd::launch_td_strings(static_cast<uint8_t*>(out_cols[idx].values), out_cols[idx].offsets,
                                        Th.SRC[idx], m[idx], static_cast<const uint8_t*>(d_rows), s);
        if (e != hipSuccess) return hip_fail(e, "td_strings");
      }
      return FORY_OK;
    }
    e = fory_amd::launch_gen_decode(G, static_cast<const uint8_t*>(d_rows), d_row_offsets, d_status, s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "gen_decode");
  }
  fory_amd::VarLaunch L{};
  rc = prepare_var(p, out_cols, num_rows, frame_mode, d_workspace, s, &L);
  if (rc) return rc;
  L.mean_row = decode_mean_row(p, L, out_cols, num_rows, frame_mode);
  e = fory_amd::launch_var_decode(L, static_cast<const uint8_t*>(d_rows), d_row_offsets, d_status, s);
  return e == hipSuccess ? FORY_OK : hip_fail(e, "var_decode");
}

int64_t fory_rowfmt_index_workspace_bytes(const fory_plan* plan, int64_t num_rows, int64_t rows_bytes) {
  if (!plan || num_rows < 0 || rows_bytes < 0) return -1;
  return align_up(fory_amd::frame_index_words(num_rows, rows_bytes, plan->p.kn.idx_frames) * 8);
}

int fory_rowfmt_index_frames(const fory_plan* plan, const void* d_rows, int64_t rows_bytes, int64_t num_rows,
                             int32_t frame_mode, int64_t* d_row_offsets, int32_t* d_status, void* d_workspace,
                             int64_t workspace_bytes, void* stream) {
  // the index overwrites the workspace: neither engine's memo survives it
  tc_forget(d_workspace);
  td_forget(d_workspace);
  if (!plan) return fail(FORY_ERR_INVALID_ARGUMENT, "plan is null");
  if (num_rows < 0 || rows_bytes < 0) return fail(FORY_ERR_INVALID_ARGUMENT, "num_rows or rows_bytes < 0");
  if (frame_mode == FORY_FRAME_RAW)
    return fail(FORY_ERR_INVALID_ARGUMENT, "raw rows are not self-delimiting: pass their row offsets to decode");
  if (frame_mode != FORY_FRAME_STREAM)
    return fail(FORY_ERR_UNSUPPORTED, "frame index: stream frames only (collection frames carry no schema hash)");
  if (!d_row_offsets) return fail(FORY_ERR_INVALID_ARGUMENT, "d_row_offsets is null");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const Plan& p = plan->p;
  hipError_t e;
  if (p.fixed_width) {  // every frame is fixed_size + 12 bytes; decode checks each size and hash
    const int64_t stride = p.fixed_size + 12;
    if (num_rows * stride > rows_bytes)
      return fail(FORY_ERR_CORRUPT, "stream holds " + std::to_string(rows_bytes) + " bytes < " +
                                        std::to_string(num_rows) + " frames x " + std::to_string(stride));
    e = fory_amd::launch_fill_offsets(d_row_offsets, num_rows, stride, s);
    return e == hipSuccess ? FORY_OK : hip_fail(e, "fill_offsets");
  }
  if (num_rows > 0 && !d_rows) return fail(FORY_ERR_INVALID_ARGUMENT, "d_rows is null");
  if (reinterpret_cast<uintptr_t>(d_rows) & 3)
    return fail(FORY_ERR_INVALID_ARGUMENT, "d_rows must be 4-byte aligned (frame starts are 4-byte aligned)");
  const int64_t need = fory_rowfmt_index_workspace_bytes(plan, num_rows, rows_bytes);
  if (num_rows > 0 && (!d_workspace || workspace_bytes < need))
    return fail(FORY_ERR_INVALID_ARGUMENT, "index workspace too small: need " + std::to_string(need) + " bytes");
  if (num_rows > 0 && rows_bytes < 12 + 8 + p.fixed_size)
    return fail(FORY_ERR_CORRUPT, "stream shorter than one frame");
  fory_amd::FrameIndexLaunch L{};
  L.rows_bytes = rows_bytes;
  L.num_rows = num_rows;
  L.schema_hash = p.schema_hash;
  L.fixed_size = p.fixed_size;
  L.idx_frames = p.kn.idx_frames;
  e = fory_amd::launch_frame_index(L, static_cast<const uint8_t*>(d_rows), d_row_offsets,
                                   static_cast<int64_t*>(d_workspace), d_status, s);
  return e == hipSuccess ? FORY_OK : hip_fail(e, "index_frames");
}

int fory_rowfmt_split_windows(const int64_t* row_offsets, int64_t stride, int64_t num_rows, int64_t max_window_bytes,
                              int32_t max_windows, int64_t* first, int32_t* num_windows) {
  if (num_rows < 0 || max_window_bytes <= 0 || max_windows <= 0 || !first || !num_windows ||
      (!row_offsets && stride <= 0))
    return fail(FORY_ERR_INVALID_ARGUMENT, "split_windows: bad arguments");
  auto at = [&](int64_t i) { return row_offsets ? row_offsets[i] : i * stride; };
  int64_t start = 0;
  int32_t w = 0;
  first[0] = 0;
  while (start < num_rows) {
    if (w == max_windows)
      return fail(FORY_ERR_CAPACITY, "more than " + std::to_string(max_windows) + " windows needed");
    const int64_t limit = at(start) + max_window_bytes;
    int64_t lo = start, hi = num_rows;  // largest e with at(e) <= limit
    while (lo < hi) {
      const int64_t mid = hi - (hi - lo) / 2;
      if (at(mid) <= limit) lo = mid;
      else hi = mid - 1;
    }
    if (lo == start)
      return fail(FORY_ERR_CAPACITY, "row " + std::to_string(start) + " (" + std::to_string(at(start + 1) - at(start)) +
                                         " bytes) exceeds a window of " + std::to_string(max_window_bytes) + " bytes");
    first[++w] = lo;
    start = lo;
  }
  *num_windows = w;
  return FORY_OK;
}

}  // extern "C"

namespace {
std::mutex g_status_words_mu;
std::vector<int32_t*> g_status_words;  // pinned status words of threads that ended
}  // namespace

extern "C" {

int fory_rowfmt_read_status(const int32_t* d_status, void* stream) {
  if (!d_status) return FORY_OK;
  // the status word lands in pinned memory of this thread (an async DMA; never the
  // runtime's pageable path): a word taken from a process-wide pool on the thread's first
  // call and handed back when the thread ends (no HIP call in a thread-exit destructor),
  // so JNI worker pools that come and go reuse words instead of pinning new ones
  struct PinnedWord {
    int32_t* p = nullptr;
    ~PinnedWord() {
      if (!p) return;
      std::lock_guard<std::mutex> lock(g_status_words_mu);
      g_status_words.push_back(p);
    }
  };
  thread_local PinnedWord word;
  if (!word.p) {
    std::lock_guard<std::mutex> lock(g_status_words_mu);
    if (!g_status_words.empty()) {
      word.p = g_status_words.back();
      g_status_words.pop_back();
    }
  }
  hipError_t e = hipSuccess;
  if (!word.p) e = hipHostMalloc(reinterpret_cast<void**>(&word.p), 64, hipHostMallocPortable | hipHostMallocCoherent);
  if (e != hipSuccess) {
    word.p = nullptr;
    return hip_fail(e, "read_status (pinned word)");
  }
  int32_t* pinned_word = word.p;
  hipStream_t s = static_cast<hipStream_t>(stream);
  *pinned_word = 0;
  e = hipMemcpyAsync(pinned_word, d_status, sizeof(int32_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return hip_fail(e, "read_status");
  const int32_t h = *pinned_word;
  switch (h) {
    case FORY_OK: return FORY_OK;
    case FORY_ERR_SCHEMA_MISMATCH:
      return fail(h, "Schema is not consistent: peer schema hash differs from this encoder's schema hash. "
                     "Please check writer schema.");
    case FORY_ERR_CORRUPT: return fail(h, "Malformed row or frame (size field out of range)");
    case FORY_ERR_CAPACITY: return fail(h, "Output buffer too small (IndexOutOfBounds)");
    case FORY_ERR_UNSUPPORTED:
      return fail(h, "BigDecimal precision cannot be greater than that in the Arrow vector "
                     "(DecimalUtility.checkPrecisionAndScale)");
    case FORY_ERR_ENCODER: return fail(h, "Encode failed (schema nesting deeper than the device stack)");
    default: return fail(h, "device status " + std::to_string(h));
  }
}

}  // extern "C"
