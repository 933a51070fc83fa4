// rv_ec.h -- the replay's coefficient-coding stage (internal): the
// committed frame's transform blocks as a coding-order job list, tokenized
// on the device (rv_ec.hip), range-coded on the host.
#pragma once

#include "rv_device.h"

namespace rv {

// the committed levels of one partition level (0 = the 64x64 superblocks)
struct EcGenLevel {
  const int32_t *l_lev = nullptr, *c_lev = nullptr;  // luma / chroma levels per block
  int n = 0, gw = 0, x0 = 0, y0 = 0;  // blocks, grid width and origin (level-block units)
  int B = 64, bc = 32;                // block size, chroma transform size (luma 64: coded 32)
};

struct EcFrameArgs {
  int tx0, ty0, tw, th, tws, ths;  // the group and the uniform tile size (superblocks)
  int xdec, ydec, ntx_c, nsb;
  const uint8_t *mi_lg, *mi_skip;  // the committed block map (luma 4x4: 4 - level, skip)
  int mi_stride, mi_cols, mi_rows;
  EcGenLevel lv[4];
  const uint64_t *words;  // result words: a superblock's winner >= 1000 is intra
  int words_per_sb, win_off;
};

struct EcFrameBufs {
  int max_jobs, ntiles, map_w4, map_h4;
  rv_ec_job *jobs;
  uint32_t *sb_off;      // [nsb + 1]
  uint8_t *map;
  void *scratch;         // rv_ec_scratch_bytes(max_jobs)
  uint32_t *offsets;     // [max_jobs + 1]
  uint32_t *tokens;      // token_cap u32 (host-mapped)
  uint32_t cap;
  uint32_t *stat;        // host-mapped [total, overflow, jobs, tile token starts [ntiles + 1]]
  uint32_t *dstat;       // device [total, overflow]
};

int ec_frame_tokens(const EcFrameArgs &a, const EcFrameBufs &b, hipStream_t st);
// worst-case jobs of a group of nsb superblocks (8x8 leaves at 4:2:0 or
// 64x64 leaves with four chroma transforms at 4:4:4)
inline int ec_max_jobs(int nsb, int ntiles) { return nsb * 194 + 2 * ntiles + 16; }

}  // namespace rv
