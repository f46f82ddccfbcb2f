// pair_seg.h -- shared between robust.hip (fa_pairwise_sqdist_rt, the tile kernels) and pairrot.hip
// (k_pairdist_rot, built without SLP vectorization so its scalar sub + fma pairs keep their DPP
// operands; see pairrot.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace fa_detail {

// one segment of the pairwise-distance input: `numel` coordinates of every client, its first chunk
// (in the launching kernel's chunk unit) and its row of client pointers in the pointer table
struct PSeg {
  int64_t numel;
  int64_t tile_start;   // first chunk of this segment (find_seg keys on it)
  int32_t ptr_base;
  int32_t pad;
  int64_t pad2;
};
static_assert(sizeof(PSeg) == 32, "PSeg layout");

constexpr int kPairRun = 64;   // longest float32 run of one pair sum (coordinates), then float64
constexpr int kRotUnit = 16;   // k_pairdist_rot: coordinates per wave step (4 rows x 4)

// k_pairdist_rot's block shape for k clients (G groups of 16, slots, waves per task set, replicas)
struct RotSplit { int G, nslots, wpt, reps, nthreads; };
RotSplit rot_split(int k);

// Launches k_pairdist_rot: nblocks workgroups, each writing the partial sums of all k(k-1)/2 pairs
// over its contiguous run of the `nunits` 16-coordinate units into partial + block * npairs.
// rt: 0 float32 differences, 1 / 2 rounded to bfloat16 / float16; vec: every client segment is
// 16-byte aligned.  Returns the hipError_t of the launch.
int launch_pairdist_rot(int k, int rt, bool vec, int nblocks, const PSeg* segs, int nseg,
                        const void* const* ptrs, int64_t nunits, double* partial, hipStream_t st);

}  // namespace fa_detail
