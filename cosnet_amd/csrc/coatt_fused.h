// Shared by the flash co-attention forward / PV kernels (coatt_fused.hip, coatt_dsplit.hip):
// tile geometry and the launch arguments (rgbd_segmentation_RAA.py:160-170, :213-221).
#pragma once
#include "common.h"

constexpr int FD = 256;              // feature channels (all_channel)
constexpr int FBQ = 128;             // query rows per workgroup
constexpr int FBK = 32;              // keys per tile
constexpr int FROWB = FD * 2;        // bytes per key row in LDS
constexpr int FTILE = FBK * FROWB;   // 16 KB per K (or V) tile
constexpr int FQB = FBQ * FROWB;     // 64 KB Q block

struct FusedDir {
  const bf16* q; const bf16* k; const bf16* v; bf16* o;
  long long ldq, ldk, ldv, ldo;
  float* lse;          // MODE 0 (optional): log2-sum-exp2 of each query row's logits x log2(e),
                       //   [B][HWp] (rows HW..HWp-1 get +inf)
  const float* klse;   // MODE 1: per-KEY normaliser in the same units, [B][HWp], +inf padded
};
struct FusedArgs {
  FusedDir dir[2];
  int HW, HWp, ndir, nrb, nwork, accumulate;
  // tail key split (MODE 0, no-grad forward).  Items = (row block, batch x direction); the
  // first nfull items run whole, one workgroup each (full rounds of the chip); each of the
  // remaining items is split over nsplit workgroups, split s covering key tiles
  // [s tps, (s+1) tps), which write their un-normalised O (fp32) and row (max, sum) to the
  // partials that coatt_merge_k folds in split order -- the last, partial round of workgroups
  // becomes a short round of short workgroups.
  int nitems, nfull, nsplit, tps;
  float* opart;    // [nsplit][nitems - nfull][128][256]
  float* mlpart;   // [nsplit][nitems - nfull][128][2]
  // coatt_q48_k (stream-K): key tiles per item, partial slots per item, per-item arrival counters
  int ntiles, smax;
  int* cnt;
};

// coatt_dsplit.hip: the d-split wave-pair variant (kernel variant 4) of the forward / PV kernel
int coatt_dsplit_launch(int mode, const FusedArgs& a, dim3 grid, hipStream_t st);

// coatt_q48.hip: 48 query rows per wave on 16x16x32 MFMA tiles (kernel variant 5), 192-row items,
// stream-K work split.  coatt_q48_launch takes a.dir / HW / HWp / accumulate; with a workspace of
// coatt_q48_workspace_bytes (and merge_ok: 16-byte output rows) it cuts items across 256
// workgroups, else it runs one workgroup per item.
int coatt_q48_rows();
size_t coatt_q48_workspace_bytes(int items, int ntiles);
int coatt_q48_launch(int mode, FusedArgs& a, int B, int nd, bool merge_ok, void* ws,
                     size_t ws_bytes, hipStream_t st);
