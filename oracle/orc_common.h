/* Internal helpers of the CPU oracle (test infrastructure only). */
#ifndef ORC_COMMON_H
#define ORC_COMMON_H

#include <stddef.h>
#include <stdint.h>

#include "rav1e_oracle.h"

/* Pixel load/store over u8/u16 buffers (Pixel trait, src/util/mod.rs:157). */
static inline int32_t orc_px(const void *p, int hbd, ptrdiff_t idx) {
  return hbd ? (int32_t)((const uint16_t *)p)[idx]
             : (int32_t)((const uint8_t *)p)[idx];
}
static inline void orc_px_store(void *p, int hbd, ptrdiff_t idx, int32_t v) {
  if (hbd)
    ((uint16_t *)p)[idx] = (uint16_t)v; /* `as u16`: truncating */
  else
    ((uint8_t *)p)[idx] = (uint8_t)v; /* `as u8`: truncating */
}

/* Wrapping i32 arithmetic (Rust release semantics). */
static inline int32_t w_add(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a + (uint32_t)b);
}
static inline int32_t w_sub(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a - (uint32_t)b);
}
static inline int32_t w_mul(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a * (uint32_t)b);
}
/* Arithmetic right shift of a signed value (gcc: `>>` on int is arithmetic). */
static inline int32_t asr(int32_t a, int b) { return a >> b; }

/* round_shift (src/util/mod.rs:241-243), wrapping add. */
static inline int32_t round_shift(int32_t v, int bit) {
  return asr(w_add(v, (1 << bit) >> 1), bit);
}

/* msb (src/util/mod.rs:235-238) */
static inline int orc_msb(int32_t x) { return 31 ^ __builtin_clz((uint32_t)x); }

static inline int32_t clamp_i32(int32_t v, int32_t lo, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}

/* TxSize geometry (src/transform/mod.rs:256-290). */
static const uint8_t ORC_TX_W_LOG2[19] = {2, 3, 4, 5, 6, 2, 3, 3, 4, 4,
                                          5, 5, 6, 2, 4, 3, 5, 4, 6};
static const uint8_t ORC_TX_H_LOG2[19] = {2, 3, 4, 5, 6, 3, 2, 4, 3, 5,
                                          4, 6, 5, 4, 2, 5, 3, 6, 4};

/* TxType -> (col kind, row kind) with kinds in TBL_IDX order
 * Id=0 Dct=1 Adst=2 FlipAdst=3 (src/transform/mod.rs:158-219). */
static const uint8_t ORC_TX_COL[16] = {1, 2, 1, 2, 3, 1, 3, 2,
                                       3, 0, 1, 0, 2, 0, 3, 0};
static const uint8_t ORC_TX_ROW[16] = {1, 1, 2, 2, 1, 3, 3, 3,
                                       2, 0, 0, 1, 0, 2, 0, 3};

#endif
