#include <stdio.h>
#include <stdlib.h>
#include <math.h>
#include "rav1e_oracle.h"
int32_t g_maxop = 0;
static unsigned long long s = 88172645463325252ull;
static unsigned rnd(void){ s ^= s<<13; s^=s>>7; s^=s<<17; return (unsigned)s; }
int main(int argc, char** argv){
  int full16 = argc > 1;
  static int16_t res[4096]; static int32_t co[4096]; static uint16_t dst[4096];
  for (int bd = 8; bd <= 12; bd += 2) {
    int m = (1<<bd)-1;
    int32_t fmax = 0, imax = 0;
    for (int ts = 0; ts < 19; ts++) for (int tt = 0; tt < 16; tt++) {
      int w = 1 << (int[]){2,3,4,5,6,2,3,3,4,4,5,5,6,2,4,3,5,4,6}[ts];
      int h = 1 << (int[]){2,3,4,5,6,3,2,4,3,5,4,6,5,4,2,5,3,6,4}[ts];
      for (int pat = 0; pat < 40; pat++) {
        int fx = rnd()%64, fy = rnd()%64;
        for (int i = 0; i < w*h; i++) {
          int r = i / w, c = i % w, v;
          if (full16) v = (int16_t)rnd();
          else if (pat < 10) v = (int)(rnd() % (2*m+1)) - m;
          else if (pat == 10) v = m; else if (pat == 11) v = -m;
          else if (pat == 12) v = ((r+c)&1) ? m : -m;
          else { double b = cos(M_PI*(2*c+1)*fx/(2.0*w)) * cos(M_PI*(2*r+1)*fy/(2.0*h)); v = b >= 0 ? m : -m; if (pat & 1) v = -v; }
          res[i] = (int16_t)v;
        }
        g_maxop = 0;
        if (orc_fwd_txfm2d(res, co, ts, tt, bd) == 0 && g_maxop > fmax) fmax = g_maxop;
        int cw = w < 32 ? w : 32, ch = h < 32 ? h : 32;
        for (int i = 0; i < cw*ch; i++) {
          int lim = 1 << (bd + 8);
          co[i] = pat < 20 ? (int)(rnd() % (2*lim+1)) - lim : ((pat&1) ? lim : -lim) * (((i + pat) & 3) ? 1 : -1);
        }
        for (int i = 0; i < w*h; i++) dst[i] = rnd() & m;
        g_maxop = 0;
        if (orc_inv_txfm2d_add(co, dst, w, ts, tt, bd, 1) == 0 && g_maxop > imax) imax = g_maxop;
      }
    }
    printf("bd %d: fwd max |mul operand| %d (log2 %.2f), inv %d (log2 %.2f)\n", bd, fmax, log2(fmax), imax, log2(imax));
  }
}
