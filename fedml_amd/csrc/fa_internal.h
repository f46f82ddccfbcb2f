// fa_internal.h -- pieces shared by the translation units of libfedagg.so (not part of the ABI):
// the context with its pinned/device staging slots, error reporting, the segment table.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "fedagg.h"

namespace fa_detail {

constexpr int kBlock = 256;
constexpr int kSlots = 8;

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// Device-resident descriptor of one state_dict tensor (staged per call from pinned host memory).
struct Seg {
  int64_t numel;
  int64_t tile_start;  // first tile (workgroup) of this segment
  void* out;
  int32_t ptr_base;    // index of client 0's pointer for this segment in the pointer table
  int32_t aligned;     // every input and the output are 16-byte aligned
};
static_assert(sizeof(Seg) == 32, "Seg layout");

// Wave-uniform lookup of the segment that owns `tile` (segments sorted by tile_start).
template <class S>
__device__ __forceinline__ int find_seg(const S* __restrict__ segs, int nseg, int64_t tile) {
  int lo = 0, hi = nseg - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (segs[mid].tile_start <= tile) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// XCD-contiguous workgroup -> tile map: the dispatcher deals workgroups to the 8 XCDs round-robin;
// XCD x then walks a contiguous eighth of the tiles (one XCD's L2 and translation caches see a few
// allocations' neighbourhoods instead of all of them)
__device__ __forceinline__ int64_t xcd_tile_map(int64_t bid, int64_t tiles) {
  constexpr int64_t kX = 8;
  const int64_t x = bid % kX, j = bid / kX, q = tiles / kX, r = tiles % kX;
  return x * q + (x < r ? x : r) + j;
}

// Record the calling thread's last error (fa_last_error) and return `code`.
int fail(int code, const char* fmt, ...);
const char* last_error();

#define FA_HIP(call)                                                                     \
  do {                                                                                   \
    hipError_t e_ = (call);                                                              \
    if (e_ != hipSuccess) return ::fa_detail::fail(FA_ERR_HIP, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) { prev = -1; }
    if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
inline bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

}  // namespace fa_detail

struct fa_ctx {
  int device = 0;
  int variant = 0;       // kernel tuning variant (results identical for every variant)
  bool mix_band = true;  // banded (sliding-window) mixing kernel when the CSR allows it
  struct Slot {
    void* host = nullptr;
    void* hmap = nullptr;  // device address of the mapped `host` buffer
    void* dev = nullptr;
    size_t cap = 0;
    hipEvent_t ev = nullptr;
    hipEvent_t staged = nullptr;  // the slot's last table copy has landed (stage())
    bool pending = false;         // FA_SLOT_EVENT=1 only: `ev` recorded at release(), host-waited
    bool ev_live = false;         // `ev` marks the end of the slot's last use (recorded at release())
    bool hit = false;             // the current use found its table already staged (stage(), reuse)
    bool copy_live = false;       // `staged` recorded and the host buffer may still be read by that copy
    hipStream_t last = nullptr;   // the stream of the slot's last use (its readers of `dev`)
    bool used = false;            // `last` is set
    std::vector<char> shadow;     // the bytes `dev` holds, for stage(..., reuse) (valid if shadow_ok)
    bool shadow_ok = false;
    bool acquired = false;        // acquire_slot'ed and not yet release()d
  } slots[fa_detail::kSlots];
  int next = 0;
  // fa_weighted_sum_host: one mapped pinned buffer the kernel reads and writes in place over PCIe
  void* zc_host = nullptr;
  void* zc_dev = nullptr;
  size_t zc_cap = 0;
  hipEvent_t zc_ev = nullptr;
  unsigned long long zc_seq = 0;  // completion word (first 256 bytes of zc_host) of the host1 path
  unsigned* zc_counter = nullptr;  // its workgroup counter (device memory)
  // fa_mt_randint_sum's jump-ahead path: per-call device work space and the jump polynomials
  void* mt_dev = nullptr;
  size_t mt_cap = 0;
  void* mt_poly_dev = nullptr;     // (count) rows of set-bit pair positions of x^(c J) mod phi, c = 1..count
  unsigned long long mt_poly_J = 0;
  int mt_poly_count = 0;
  int mt_poly_stride = 0;
  hipEvent_t mt_ev = nullptr;  // the last jump-path call's kernels have finished with mt_dev / mt_poly_dev
  bool mt_live = false;        // mt_ev has been recorded
};

namespace fa_detail {

// Take the next staging slot with >= bytes of room.  The host waits only for a table copy still
// reading the slot's host buffer (a copy kSlots calls ago); the slot's earlier kernels are ordered
// before a later copy into its device buffer on the device (stage()), with no per-call event.
int acquire_slot(fa_ctx* ctx, size_t bytes, fa_ctx::Slot** out);
// Copy the slot's first `bytes` host bytes to its device buffer (async on `st`).
// reuse: the caller's kernels only READ the table; if the slot's device buffer already holds exactly
// these bytes (the same table staged through this slot before), the copy -- and the caller stream's
// wait for it -- is skipped.
int stage(fa_ctx::Slot* s, size_t bytes, hipStream_t st, bool reuse = false);
// End of the slot's use by the work queued on `st` (stage() orders a later copy after it).
int release(fa_ctx::Slot* s, hipStream_t st);

}  // namespace fa_detail
