#include "orc_common.h"
extern int32_t g_maxop;
static inline int32_t w_mul_chk(int32_t a, int32_t b) {
  int32_t x = (a < 0 ? -a : a) > (b < 0 ? -b : b) ? a : b; /* the data operand */
  int32_t ax = x < 0 ? -x : x;
  if (ax > g_maxop) g_maxop = ax;
  return (int32_t)((uint32_t)a * (uint32_t)b);
}
#define w_mul(a, b) w_mul_chk(a, b)
