/* Forward transform restatement (test infrastructure only).
 *
 * Follows src/transform/forward.rs: the Daala integer-lifting DCT-II /
 * DST-IV / DST-VII kernels (:100-1700) and the 2-D driver FwdTxfm2D::fht
 * (:1804-1899).  All lanes of the reference's SIMD types are independent,
 * so the scalar form here is lane-for-lane identical; i32 ops wrap.
 *
 * Structure note: every daala_fdct_ii_N (N = 8, 16, 32, 64; :468, :689,
 * :1072, :1551) and daala_fdct_ii_N_asym (:421, :617, :917, :1212) uses the
 * same even/odd butterfly pattern and recurses into the N/2 DCT plus an
 * N/2 DST-IV whose outputs are stored reversed; that shared pattern is
 * written once below (fdct_ii / fdct_ii_asym).  The DST-IV kernels carry
 * size-specific constants and are restated one by one.
 */
#include <string.h>

#include "orc_common.h"

typedef int32_t T;
typedef struct { T h, f; } P2; /* (half, full) tuple of the reference */
typedef struct { T a, b; } TT; /* plain 2-tuple result */

/* TxOperations for i32, forward.rs:114-130 */
static inline T txmul(T x, int m, int s) {
  return asr(w_add(w_mul(x, m), (1 << s) >> 1), s);
}
static inline T rsh1(T x) { return asr(w_add(x, x < 0 ? 1 : 0), 1); }
static inline T add_avg(T a, T b) { return asr(w_add(a, b), 1); }
static inline T sub_avg(T a, T b) { return asr(w_sub(a, b), 1); }
#define ADD w_add
#define SUB w_sub

/* RotateKernelPi4 (forward.rs:164-199). kind: 0 Add, 1 AddAvg, 2 Sub,
 * 3 SubAvg. */
static TT rot_pi4(int kind, T p0, T p1, int m0, int s0, int m1, int s1) {
  T t;
  switch (kind) {
  case 0: t = ADD(p1, p0); break;
  case 1: t = add_avg(p1, p0); break;
  case 2: t = SUB(p1, p0); break;
  default: t = sub_avg(p1, p0); break;
  }
  T a = txmul(p0, m0, s0);
  T out0 = txmul(t, m1, s1);
  T out1 = kind < 2 ? SUB(a, out0) : ADD(a, out0);
  TT r = {out0, out1};
  return r;
}

/* RotateKernel::half_kernel (forward.rs:201-277). */
enum { RADD, RADDAVG, RADDSHIFT, RSUB, RSUBAVG, RSUBSHIFT };
static TT rot_half(int kind, P2 p0, T p1, int m0, int s0, int m1, int s1,
                   int m2, int s2) {
  T t;
  switch (kind) {
  case RADD:
  case RADDSHIFT: t = ADD(p1, p0.h); break;
  case RADDAVG: t = add_avg(p1, p0.h); break;
  case RSUB:
  case RSUBSHIFT: t = SUB(p1, p0.h); break;
  default: t = sub_avg(p1, p0.h); break;
  }
  T a = txmul(p0.f, m0, s0), b = txmul(p1, m1, s1), c = txmul(t, m2, s2);
  T out0 = ADD(b, c);
  T sh = (kind == RADDSHIFT || kind == RSUBSHIFT) ? rsh1(c) : c;
  T out1 = kind <= RADDSHIFT ? SUB(a, sh) : ADD(a, sh);
  TT r = {out0, out1};
  return r;
}
static inline TT rot(int kind, T p0, T p1, int m0, int s0, int m1, int s1,
                     int m2, int s2) {
  P2 p = {p0, p0};
  return rot_half(kind, p, p1, m0, s0, m1, s1, m2, s2);
}
/* RotateKernelNeg (forward.rs:222-285): avg = 0 RotateNeg, 1 RotateNegAvg */
static TT rot_neg(int avg, T p0, T p1, int m0, int s0, int m1, int s1, int m2,
                  int s2) {
  T t = avg ? sub_avg(p0, p1) : SUB(p0, p1);
  T a = txmul(p0, m0, s0), b = txmul(p1, m1, s1), c = txmul(t, m2, s2);
  TT r = {SUB(b, c), SUB(c, a)};
  return r;
}

/* Butterflies, forward.rs:287-324 */
static inline void bf_add(T p0, T p1, P2 *o0, T *o1h) {
  T s = ADD(p0, p1);
  T sh = rsh1(s);
  o0->h = sh;
  o0->f = s;
  *o1h = SUB(p1, sh);
}
static inline void bf_sub(T p0, T p1, P2 *o0, T *o1h) {
  T s = SUB(p0, p1);
  T sh = rsh1(s);
  o0->h = sh;
  o0->f = s;
  *o1h = ADD(p1, sh);
}
static inline void bf_neg(T p0, T p1, T *o0h, P2 *o1) {
  T d = SUB(p0, p1);
  T dh = rsh1(d);
  *o0h = SUB(p0, dh);
  o1->h = dh;
  o1->f = d;
}
static inline TT bf_add_asym(P2 p0, T p1h) {
  T p1 = ADD(p1h, p0.h);
  TT r = {SUB(p0.f, p1), p1};
  return r;
}
static inline TT bf_sub_asym(P2 p0, T p1h) {
  T p1 = SUB(p1h, p0.h);
  TT r = {ADD(p0.f, p1), p1};
  return r;
}
static inline TT bf_neg_asym(T p0h, P2 p1) {
  T p0 = ADD(p0h, p1.h);
  TT r = {p0, SUB(p0, p1.f)};
  return r;
}
static inline P2 hp(T x) { /* (x.rshift1(), x) */
  P2 p = {rsh1(x), x};
  return p;
}

#define SET(x, y, expr) \
  do {                  \
    TT r_ = (expr);     \
    x = r_.a;           \
    y = r_.b;           \
  } while (0)

/* ---- 2-point and 4-point kernels ------------------------------------- */

/* daala_fdct_ii_2 (forward.rs:407-412) */
static TT fdct_ii_2(T p0, T p1) {
  TT r = rot_pi4(3, p1, p0, 11585, 13, 11585, 13); /* (p1, p0) */
  TT o = {r.b, r.a};
  return o;
}
/* daala_fdst_iv_2 (forward.rs:414-419) */
static TT fdst_iv_2(T p0, T p1) {
  return rot(RADDAVG, p0, p1, 10703, 13, 8867, 14, 3135, 12);
}
/* daala_fdst_iv_2_asym (forward.rs:342-347) */
static TT fdst_iv_2_asym(P2 p0, T p1h) {
  return rot_half(RADD, p0, p1h, 473, 9, 3135, 12, 4433, 13);
}

/* daala_fdst_iv_4 (forward.rs:590-615) */
static void fdst_iv_4(const T *in, T *out) {
  T q0 = in[0], q1 = in[1], q2 = in[2], q3 = in[3];
  SET(q0, q3, rot(RADDSHIFT, q0, q3, 13623, 14, 4551, 12, 565, 11));
  SET(q2, q1, rot(RSUBSHIFT, q2, q1, 16069, 14, 12785, 15, 1609, 11));
  SET(q2, q3, bf_sub_asym(hp(q2), q3));
  SET(q0, q1, bf_sub_asym(hp(q0), q1));
  SET(q2, q1, rot_pi4(1, q2, q1, 11585, 13, 11585, 13));
  out[0] = q0; out[1] = q1; out[2] = q2; out[3] = q3;
}

/* daala_fdst_iv_4_asym (forward.rs:435-466); args q0:P2 q1h q2:P2 q3h */
static void fdst_iv_4_asym(const P2 *pp, const T *hh, T *out) {
  T q0, q1, q2, q3;
  SET(q0, q3, rot_half(RADDSHIFT, pp[0], hh[3], 9633, 14, 12873, 13, 12785,
                       15));
  SET(q2, q1, rot_half(RSUBSHIFT, pp[2], hh[1], 11363, 14, 18081, 15, 4551,
                       12));
  SET(q2, q3, bf_sub_asym(hp(q2), q3));
  SET(q0, q1, bf_sub_asym(hp(q0), q1));
  SET(q2, q1, rot_pi4(1, q2, q1, 11585, 13, 11585, 13));
  out[0] = q0; out[1] = q1; out[2] = q2; out[3] = q3;
}

/* ---- 8-point DST-IV kernels ----------------------------------------- */

/* daala_fdst_iv_8 (forward.rs:509-562) */
static void fdst_iv_8(const T *in, T *out) {
  T r0 = in[0], r1 = in[1], r2 = in[2], r3 = in[3], r4 = in[4], r5 = in[5],
    r6 = in[6], r7 = in[7];
  SET(r0, r7, rot(RADD, r0, r7, 17911, 14, 14699, 14, 803, 13));
  SET(r6, r1, rot(RSUB, r6, r1, 20435, 14, 21845, 15, 1189, 12));
  SET(r2, r5, rot(RADD, r2, r5, 22173, 14, 3363, 13, 15447, 15));
  SET(r4, r3, rot(RSUB, r4, r3, 23059, 14, 2271, 14, 5197, 13));
  P2 R0, R2, R5, R7;
  T r3h, r1h, r6h, r4h;
  bf_add(r0, r3, &R0, &r3h);
  bf_sub(r2, r1, &R2, &r1h);
  bf_add(r5, r6, &R5, &r6h);
  bf_sub(r7, r4, &R7, &r4h);
  SET(r7, r6, bf_add_asym(R7, r6h));
  SET(r5, r3, bf_add_asym(R5, r3h));
  SET(r2, r4, bf_add_asym(R2, r4h));
  SET(r0, r1, bf_sub_asym(R0, r1h));
  SET(r3, r4, rot(RSUBAVG, r3, r4, 10703, 13, 8867, 14, 3135, 12));
  SET(r2, r5, rot_neg(1, r2, r5, 10703, 13, 8867, 14, 3135, 12));
  SET(r1, r6, rot_pi4(3, r1, r6, 11585, 13, 11585, 13));
  out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3;
  out[4] = r4; out[5] = r5; out[6] = r6; out[7] = r7;
}

/* daala_fdst_iv_8_asym (forward.rs:633-687); args r0:P2 r1h r2:P2 ... r7h */
static void fdst_iv_8_asym(const P2 *pp, const T *hh, T *out) {
  T r0, r1, r2, r3, r4, r5, r6, r7;
  SET(r0, r7, rot_half(RADD, pp[0], hh[7], 12665, 14, 5197, 12, 2271, 14));
  SET(r6, r1, rot_half(RSUB, pp[6], hh[1], 14449, 14, 30893, 15, 3363, 13));
  SET(r2, r5, rot_half(RADD, pp[2], hh[5], 15679, 14, 1189, 11, 5461, 13));
  SET(r4, r3, rot_half(RSUB, pp[4], hh[3], 16305, 14, 803, 12, 14699, 14));
  P2 R0, R2, R5, R7;
  T r3h, r1h, r6h, r4h;
  bf_add(r0, r3, &R0, &r3h);
  bf_sub(r2, r1, &R2, &r1h);
  bf_add(r5, r6, &R5, &r6h);
  bf_sub(r7, r4, &R7, &r4h);
  SET(r7, r6, bf_add_asym(R7, r6h));
  SET(r5, r3, bf_add_asym(R5, r3h));
  SET(r2, r4, bf_add_asym(R2, r4h));
  SET(r0, r1, bf_sub_asym(R0, r1h));
  SET(r3, r4, rot(RSUBAVG, r3, r4, 669, 9, 8867, 14, 3135, 12));
  SET(r2, r5, rot_neg(1, r2, r5, 669, 9, 8867, 14, 3135, 12));
  SET(r1, r6, rot_pi4(3, r1, r6, 5793, 12, 11585, 13));
  out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3;
  out[4] = r4; out[5] = r5; out[6] = r6; out[7] = r7;
}

/* ---- 16-point DST-IV kernels ---------------------------------------- */
/* Index names follow the reference: s0..s9 = 0..9, sa..sf = 10..15. */

/* Stages 1, 2 and 4 shared by daala_fdst_iv_16 (:797-847) and
 * daala_fdst_iv_16_asym (:994-1044); stage 3 differs and is passed in. */
typedef void (*stage3_fn)(T *s, T s9h, T s6h, T s4h, T sbh);

static void fdst16_core(T *s, stage3_fn stage3, int stage5_asym) {
  P2 S0, S2, Sd, Sf;
  T s3h, seh, s1h, sch, s4h, sbh, s6h, s9h, dummy;
  P2 Ptmp;
  /* Stage 1 */
  SET(s[0], s[7], bf_sub_asym(hp(s[0]), s[7]));
  SET(s[8], s[15], bf_sub_asym(hp(s[8]), s[15]));
  SET(s[4], s[3], bf_add_asym(hp(s[4]), s[3]));
  SET(s[12], s[11], bf_add_asym(hp(s[12]), s[11]));
  SET(s[2], s[5], bf_sub_asym(hp(s[2]), s[5]));
  SET(s[10], s[13], bf_sub_asym(hp(s[10]), s[13]));
  SET(s[6], s[1], bf_add_asym(hp(s[6]), s[1]));
  SET(s[14], s[9], bf_add_asym(hp(s[14]), s[9]));
  /* Stage 2 */
  bf_add(s[8], s[4], &Ptmp, &s4h);
  s[8] = Ptmp.f;
  bf_add(s[7], s[11], &Ptmp, &sbh);
  s[7] = Ptmp.f;
  bf_sub(s[10], s[6], &Ptmp, &s6h);
  s[10] = Ptmp.f;
  bf_sub(s[5], s[9], &Ptmp, &s9h);
  s[5] = Ptmp.f;
  bf_add(s[0], s[3], &S0, &s3h);
  bf_add(s[13], s[14], &Sd, &seh);
  bf_sub(s[2], s[1], &S2, &s1h);
  bf_sub(s[15], s[12], &Sf, &sch);
  (void)dummy;
  /* Stage 3 */
  stage3(s, s9h, s6h, s4h, sbh);
  /* Stage 4 */
  SET(s[2], s[12], bf_add_asym(S2, sch));
  SET(s[0], s[1], bf_sub_asym(S0, s1h));
  SET(s[15], s[14], bf_add_asym(Sf, seh));
  SET(s[13], s[3], bf_add_asym(Sd, s3h));
  SET(s[7], s[6], bf_add_asym(hp(s[7]), s[6]));
  SET(s[8], s[9], bf_sub_asym(hp(s[8]), s[9]));
  SET(s[10], s[11], bf_sub_asym(hp(s[10]), s[11]));
  SET(s[5], s[4], bf_add_asym(hp(s[5]), s[4]));
  /* Stage 5 */
  if (!stage5_asym) { /* forward.rs:850-868 */
    SET(s[12], s[3], rot(RADDAVG, s[12], s[3], 669, 9, 8867, 14, 3135, 12));
    SET(s[2], s[13], rot_neg(1, s[2], s[13], 669, 9, 8867, 14, 3135, 12));
    SET(s[10], s[5], rot_pi4(1, s[10], s[5], 5793, 12, 11585, 13));
    SET(s[6], s[9], rot_pi4(1, s[6], s[9], 5793, 12, 11585, 13));
    SET(s[14], s[1], rot_pi4(1, s[14], s[1], 5793, 12, 11585, 13));
  } else { /* forward.rs:1047-1065 */
    SET(s[12], s[3], rot(RADD, s[12], s[3], 10703, 13, 8867, 14, 3135, 13));
    SET(s[2], s[13], rot_neg(0, s[2], s[13], 10703, 13, 8867, 14, 3135, 13));
    SET(s[10], s[5], rot_pi4(0, s[10], s[5], 11585, 13, 5793, 13));
    SET(s[6], s[9], rot_pi4(0, s[6], s[9], 11585, 13, 5793, 13));
    SET(s[14], s[1], rot_pi4(0, s[14], s[1], 11585, 13, 5793, 13));
  }
}

/* Stage 3 of daala_fdst_iv_16, forward.rs:818-837 */
static void fdst16_stage3(T *s, T s9h, T s6h, T s4h, T sbh) {
  SET(s[8], s[7], rot(RADDAVG, s[8], s[7], 301, 8, 1609, 11, 12785, 15));
  SET(s[9], s[6], rot(RADD, s9h, s6h, 11363, 13, 9041, 15, 4551, 13));
  SET(s[5], s[10], rot_neg(1, s[5], s[10], 5681, 12, 9041, 15, 4551, 12));
  SET(s[4], s[11], rot_neg(0, s4h, sbh, 9633, 13, 12873, 14, 6393, 15));
}
/* Stage 3 of daala_fdst_iv_16_asym, forward.rs:1015-1034 */
static void fdst16a_stage3(T *s, T s9h, T s6h, T s4h, T sbh) {
  SET(s[8], s[7], rot(RADD, s[8], s[7], 9633, 13, 12873, 14, 6393, 15));
  SET(s[9], s[6], rot(RADD, s9h, s6h, 22725, 14, 9041, 15, 4551, 13));
  SET(s[5], s[10], rot_neg(0, s[5], s[10], 11363, 13, 9041, 15, 4551, 13));
  SET(s[4], s[11], rot_neg(0, s4h, sbh, 9633, 13, 12873, 14, 6393, 15));
}

/* daala_fdst_iv_16, forward.rs:751-873 */
static void fdst_iv_16(const T *in, T *out) {
  T s[16];
  memcpy(s, in, sizeof(s));
  SET(s[0], s[15], rot(RADDSHIFT, s[0], s[15], 24279, 15, 11003, 13, 1137, 14));
  SET(s[14], s[1], rot(RSUBSHIFT, s[14], s[1], 1645, 11, 305, 8, 425, 11));
  SET(s[2], s[13], rot(RADDSHIFT, s[2], s[13], 14053, 14, 8423, 13, 2815, 13));
  SET(s[12], s[3], rot(RSUBSHIFT, s[12], s[3], 14811, 14, 7005, 13, 3903, 13));
  SET(s[4], s[11], rot(RADDSHIFT, s[4], s[11], 30853, 15, 11039, 14, 9907, 14));
  SET(s[10], s[5], rot(RSUBSHIFT, s[10], s[5], 15893, 14, 3981, 13, 1489, 11));
  SET(s[6], s[9], rot(RADDSHIFT, s[6], s[9], 32413, 15, 601, 11, 13803, 14));
  SET(s[8], s[7], rot(RSUBSHIFT, s[8], s[7], 32729, 15, 201, 11, 1945, 11));
  fdst16_core(s, fdst16_stage3, 0);
  memcpy(out, s, sizeof(s));
}

/* daala_fdst_iv_16_asym, forward.rs:938-1070; args s0:P2 s1h s2:P2 ... */
static void fdst_iv_16_asym(const P2 *pp, const T *hh, T *out) {
  T s[16];
  SET(s[0], s[15], rot_half(RADDSHIFT, pp[0], hh[15], 1073, 11, 62241, 15,
                            201, 11));
  SET(s[14], s[1], rot_half(RSUBSHIFT, pp[14], hh[1], 18611, 15, 55211, 15,
                            601, 11));
  SET(s[2], s[13], rot_half(RADDSHIFT, pp[2], hh[13], 9937, 14, 1489, 10,
                            3981, 13));
  SET(s[12], s[3], rot_half(RSUBSHIFT, pp[12], hh[3], 10473, 14, 39627, 15,
                            11039, 14));
  SET(s[4], s[11], rot_half(RADDSHIFT, pp[4], hh[11], 2727, 12, 3903, 12,
                            7005, 13));
  SET(s[10], s[5], rot_half(RSUBSHIFT, pp[10], hh[5], 5619, 13, 2815, 12,
                            8423, 13));
  /* the reference uses 13599 here (its comment says 13588), forward.rs:984 */
  SET(s[6], s[9], rot_half(RADDSHIFT, pp[6], hh[9], 2865, 12, 13599, 15, 305,
                           8));
  SET(s[8], s[7], rot_half(RSUBSHIFT, pp[8], hh[7], 23143, 15, 1137, 13,
                           11003, 13));
  fdst16_core(s, fdst16a_stage3, 1);
  memcpy(out, s, sizeof(s));
}

/* ---- 32-point DST-IV (asymmetric input), forward.rs:1279-1548 -------- */
/* Names: t0..t9 = 0..9, ta..tv = 10..31. */
static void fdst_iv_32_asym(const P2 *pp, const T *hh, T *out) {
  T t[32];
  /* Stage 0 */
  SET(t[0], t[31], rot_half(RADD, pp[0], hh[31], 5933, 13, 22595, 14, 1137, 15));
  SET(t[30], t[1], rot_half(RSUB, pp[30], hh[1], 6203, 13, 21403, 14, 3409, 15));
  SET(t[2], t[29], rot_half(RADD, pp[2], hh[29], 25833, 15, 315, 8, 5673, 15));
  SET(t[28], t[3], rot_half(RSUB, pp[28], hh[3], 26791, 15, 4717, 12, 7923, 15));
  SET(t[4], t[27], rot_half(RADD, pp[4], hh[27], 6921, 13, 17531, 14, 10153, 15));
  SET(t[26], t[5], rot_half(RSUB, pp[26], hh[5], 28511, 15, 32303, 15, 1545, 12));
  SET(t[6], t[25], rot_half(RADD, pp[6], hh[25], 29269, 15, 14733, 14, 1817, 12));
  SET(t[24], t[7], rot_half(RSUB, pp[24], hh[7], 29957, 15, 13279, 14, 8339, 14));
  SET(t[8], t[23], rot_half(RADD, pp[8], hh[23], 7643, 13, 11793, 14, 18779, 15));
  SET(t[22], t[9], rot_half(RSUB, pp[22], hh[9], 15557, 14, 20557, 15, 20835, 15));
  SET(t[10], t[21], rot_half(RADD, pp[10], hh[21], 31581, 15, 17479, 15, 22841, 15));
  SET(t[20], t[11], rot_half(RSUB, pp[20], hh[11], 7993, 13, 14359, 15, 3099, 12));
  SET(t[12], t[19], rot_half(RADD, pp[12], hh[19], 16143, 14, 2801, 13, 26683, 15));
  SET(t[18], t[13], rot_half(RSUB, pp[18], hh[13], 16261, 14, 4011, 14, 14255, 14));
  SET(t[14], t[17], rot_half(RADD, pp[14], hh[17], 32679, 15, 4821, 15, 30269, 15));
  SET(t[16], t[15], rot_half(RSUB, pp[16], hh[15], 16379, 14, 201, 12, 15977, 14));

  /* Stage 1 (:1369-1384): pairs P[x] and halves H[x] by index */
  P2 P[32];
  T H[32];
  bf_add(t[0], t[15], &P[0], &H[15]);
  bf_sub(t[31], t[16], &P[31], &H[16]);
  bf_add(t[17], t[30], &P[17], &H[30]);
  bf_sub(t[14], t[1], &P[14], &H[1]);
  bf_add(t[2], t[13], &P[2], &H[13]);
  bf_sub(t[29], t[18], &P[29], &H[18]);
  bf_add(t[19], t[28], &P[19], &H[28]);
  bf_sub(t[12], t[3], &P[12], &H[3]);
  bf_add(t[4], t[11], &P[4], &H[11]);
  bf_sub(t[27], t[20], &P[27], &H[20]);
  bf_add(t[21], t[26], &P[21], &H[26]);
  bf_sub(t[10], t[5], &P[10], &H[5]);
  bf_add(t[6], t[9], &P[6], &H[9]);
  bf_sub(t[25], t[22], &P[25], &H[22]);
  bf_add(t[23], t[24], &P[23], &H[24]);
  bf_sub(t[8], t[7], &P[8], &H[7]);

  /* Stage 2 (:1387-1402) */
  SET(t[0], t[7], bf_sub_asym(P[0], H[7]));
  SET(t[31], t[24], bf_add_asym(P[31], H[24]));
  SET(t[25], t[30], bf_sub_asym(P[25], H[30]));
  SET(t[6], t[1], bf_add_asym(P[6], H[1]));
  SET(t[2], t[5], bf_sub_asym(P[2], H[5]));
  SET(t[29], t[26], bf_add_asym(P[29], H[26]));
  SET(t[27], t[28], bf_sub_asym(P[27], H[28]));
  SET(t[4], t[3], bf_add_asym(P[4], H[3]));
  SET(t[8], t[16], bf_add_asym(P[8], H[16]));
  SET(t[14], t[22], bf_sub_asym(P[14], H[22]));
  SET(t[23], t[15], bf_add_asym(P[23], H[15]));
  SET(t[17], t[9], bf_sub_asym(P[17], H[9]));
  SET(t[10], t[18], bf_add_asym(P[10], H[18]));
  SET(t[12], t[20], bf_sub_asym(P[12], H[20]));
  SET(t[21], t[13], bf_add_asym(P[21], H[13]));
  SET(t[19], t[11], bf_sub_asym(P[19], H[11]));

  /* Stage 3 (:1408-1444) */
  SET(t[15], t[16], rot(RSUB, t[15], t[16], 17911, 14, 14699, 14, 803, 13));
  SET(t[17], t[14], rot(RADD, t[17], t[14], 10217, 13, 5461, 13, 1189, 12));
  SET(t[18], t[13], rot(RADD, t[18], t[13], 5543, 12, 3363, 13, 7723, 14));
  SET(t[12], t[19], rot(RSUB, t[12], t[19], 11529, 13, 2271, 14, 5197, 13));
  SET(t[11], t[20], rot_neg(0, t[11], t[20], 11529, 13, 2271, 14, 5197, 13));
  SET(t[10], t[21], rot_neg(0, t[10], t[21], 5543, 12, 3363, 13, 7723, 14));
  SET(t[9], t[22], rot_neg(0, t[9], t[22], 10217, 13, 5461, 13, 1189, 12));
  SET(t[8], t[23], rot_neg(0, t[8], t[23], 17911, 14, 14699, 14, 803, 13));

  /* Stage 4 (:1447-1462) */
  P2 Q[32];
  T G[32];
  bf_sub(t[3], t[0], &Q[3], &G[0]);
  bf_add(t[28], t[31], &Q[28], &G[31]);
  bf_sub(t[30], t[29], &Q[30], &G[29]);
  bf_add(t[1], t[2], &Q[1], &G[2]);
  bf_add(t[24], t[4], &Q[24], &G[4]);
  bf_sub(t[26], t[6], &Q[26], &G[6]);
  bf_add(t[7], t[27], &Q[7], &G[27]);
  bf_sub(t[5], t[25], &Q[5], &G[25]);
  bf_sub(t[11], t[8], &Q[11], &G[8]);
  bf_add(t[20], t[23], &Q[20], &G[23]);
  bf_sub(t[22], t[21], &Q[22], &G[21]);
  bf_add(t[9], t[10], &Q[9], &G[10]);
  bf_sub(t[15], t[12], &Q[15], &G[12]);
  bf_add(t[16], t[19], &Q[16], &G[19]);
  bf_sub(t[18], t[17], &Q[18], &G[17]);
  bf_add(t[13], t[14], &Q[13], &G[14]);
  /* to, tq, t7, t5 only keep their full value (:1451-1454) */
  t[24] = Q[24].f;
  t[26] = Q[26].f;
  t[7] = Q[7].f;
  t[5] = Q[5].f;

  /* Stage 5 (:1468-1483) */
  SET(t[24], t[7], rot(RADD, t[24], t[7], 301, 8, 1609, 11, 6393, 15));
  SET(G[25], G[6], rot(RADD, G[25], G[6], 11363, 13, 9041, 15, 4551, 13));
  SET(t[5], t[26], rot_neg(0, t[5], t[26], 5681, 12, 9041, 15, 4551, 13));
  SET(G[4], G[27], rot_neg(0, G[4], G[27], 9633, 13, 12873, 14, 6393, 15));

  /* Stage 6 (:1486-1501) */
  SET(t[1], t[0], bf_add_asym(Q[1], G[0]));
  SET(t[30], t[31], bf_sub_asym(Q[30], G[31]));
  SET(t[28], t[2], bf_sub_asym(Q[28], G[2]));
  SET(t[3], t[29], bf_sub_asym(Q[3], G[29]));
  SET(t[5], t[4], bf_add_asym(hp(t[5]), G[4]));
  SET(t[26], t[27], bf_sub_asym(hp(t[26]), G[27]));
  SET(t[7], t[6], bf_add_asym(hp(t[7]), G[6]));
  SET(t[24], t[25], bf_sub_asym(hp(t[24]), G[25]));
  SET(t[9], t[8], bf_add_asym(Q[9], G[8]));
  SET(t[22], t[23], bf_sub_asym(Q[22], G[23]));
  SET(t[20], t[10], bf_sub_asym(Q[20], G[10]));
  SET(t[11], t[21], bf_sub_asym(Q[11], G[21]));
  SET(t[18], t[12], bf_add_asym(Q[18], G[12]));
  SET(t[13], t[19], bf_add_asym(Q[13], G[19]));
  SET(t[15], t[14], bf_add_asym(Q[15], G[14]));
  SET(t[16], t[17], bf_sub_asym(Q[16], G[17]));

  /* Stage 7 (:1507-1542) */
  SET(t[2], t[29], rot_neg(0, t[2], t[29], 669, 9, 8867, 14, 3135, 13));
  SET(t[28], t[3], rot(RADD, t[28], t[3], 669, 9, 8867, 14, 3135, 13));
  SET(t[10], t[21], rot_neg(0, t[10], t[21], 669, 9, 8867, 14, 3135, 13));
  SET(t[20], t[11], rot(RADD, t[20], t[11], 669, 9, 8867, 14, 3135, 13));
  SET(t[12], t[19], rot(RADD, t[12], t[19], 669, 9, 8867, 14, 3135, 13));
  SET(t[18], t[13], rot_neg(0, t[18], t[13], 669, 9, 8867, 14, 3135, 13));
  SET(t[30], t[1], rot_pi4(0, t[30], t[1], 5793, 12, 5793, 13));
  SET(t[26], t[5], rot_pi4(0, t[26], t[5], 5793, 12, 5793, 13));
  SET(t[25], t[6], rot_pi4(2, t[25], t[6], 5793, 12, 5793, 13));
  SET(t[22], t[9], rot_pi4(0, t[22], t[9], 5793, 12, 5793, 13));
  SET(t[14], t[17], rot_pi4(0, t[14], t[17], 5793, 12, 5793, 13));
  memcpy(out, t, sizeof(t));
}

/* ---- generic DCT-II recursion ---------------------------------------- */

static void fdct_ii(int n, const T *x, T *out);

/* daala_fdct_ii_N_asym, N = 4, 8, 16, 32 (forward.rs:421-433, 617-631,
 * 917-936, 1212-1277): even inputs are halves, odd inputs are pairs. */
static void fdct_ii_asym(int n, const T *hh, const P2 *pp, T *out) {
  T x[32];
  for (int i = 0; i < n / 2; i++) {
    int j = n - 1 - i;
    TT r = (i & 1) ? bf_sub_asym(pp[i], hh[j]) : bf_neg_asym(hh[i], pp[j]);
    x[i] = r.a;
    x[j] = r.b;
  }
  T lo[32], hi[32], rev[32];
  int m = n / 2;
  for (int k = 0; k < m; k++) rev[k] = x[n - 1 - k];
  if (n == 4) {
    TT a = fdct_ii_2(x[0], x[1]);
    TT b = fdst_iv_2(rev[0], rev[1]);
    lo[0] = a.a; lo[1] = a.b;
    hi[0] = b.a; hi[1] = b.b;
  } else {
    fdct_ii(m, x, lo);
    if (m == 4) fdst_iv_4(rev, hi);
    else if (m == 8) fdst_iv_8(rev, hi);
    else fdst_iv_16(rev, hi);
  }
  for (int k = 0; k < m; k++) {
    out[k] = lo[k];
    out[m + k] = hi[m - 1 - k];
  }
}

/* daala_fdct_ii_N, N = 4, 8, 16, 32, 64 (forward.rs:349-361, 468-481,
 * 689-707, 1072-1136, 1551-1658). */
static void fdct_ii(int n, const T *x, T *out) {
  T hh[64];
  P2 pp[64];
  for (int i = 0; i < n / 2; i++) {
    int j = n - 1 - i;
    if (i & 1) bf_add(x[i], x[j], &pp[i], &hh[j]);
    else bf_neg(x[i], x[j], &hh[i], &pp[j]);
  }
  int m = n / 2;
  T lo[32], hi[32];
  /* the DST half receives (P[n-1], H[n-2], P[n-3], ...) */
  P2 dp[32] = {{0, 0}};
  T dh[32] = {0};
  for (int k = 0; k < m; k++) {
    if (k & 1) dh[k] = hh[n - 1 - k];
    else dp[k] = pp[n - 1 - k];
  }
  if (n == 4) {
    TT a = bf_neg_asym(hh[0], pp[1]); /* daala_fdct_ii_2_asym */
    TT b = fdst_iv_2_asym(dp[0], dh[1]);
    lo[0] = a.a; lo[1] = a.b;
    hi[0] = b.a; hi[1] = b.b;
  } else {
    fdct_ii_asym(m, hh, pp, lo);
    if (m == 4) fdst_iv_4_asym(dp, dh, hi);
    else if (m == 8) fdst_iv_8_asym(dp, dh, hi);
    else if (m == 16) fdst_iv_16_asym(dp, dh, hi);
    else fdst_iv_32_asym(dp, dh, hi);
  }
  for (int k = 0; k < m; k++) {
    out[k] = lo[k];
    out[m + k] = hi[m - 1 - k];
  }
}

static inline int brev(int bits, int x) {
  int r = 0;
  for (int i = 0; i < bits; i++) r |= ((x >> i) & 1) << (bits - 1 - i);
  return r;
}

/* daala_fdst_vii_4 (forward.rs:375-405) */
static void fdst_vii_4(const T *in, T *out) {
  T q0 = in[0], q1 = in[1], q2 = in[2], q3 = in[3];
  T t0 = ADD(q1, q3);
  T t1 = ADD(q1, sub_avg(q0, t0));
  T t2 = SUB(q0, q1);
  T t3 = q2;
  T t4 = ADD(q0, q3);
  t0 = txmul(t0, 7021, 14);
  t1 = txmul(t1, 37837, 15);
  t2 = txmul(t2, 21513, 15);
  t3 = txmul(t3, 37837, 15);
  t4 = txmul(t4, 467, 11);
  T t3h = rsh1(t3);
  T u4 = ADD(t4, t3h);
  out[0] = ADD(t0, u4);
  out[1] = t1;
  out[2] = ADD(t0, SUB(t2, t3h));
  out[3] = ADD(t2, SUB(t3, u4));
}

/* txfm_types::Detail::forward dispatch (forward.rs:1745-1768). */
int orc_fwd_txfm1d(int kind, int n, const int32_t *in, int32_t *out) {
  int lg = n == 4 ? 2 : n == 8 ? 3 : n == 16 ? 4 : n == 32 ? 5 : n == 64 ? 6 : 0;
  if (!lg) return -1;
  T tmp[64];
  switch (kind) {
  case 0: /* Id: fidentity4..32, no Id64 */
    if (n == 64) return -1;
    memcpy(out, in, (size_t)n * sizeof(T));
    return 0;
  case 1: /* Dct: daala_fdct4..64 = bit-reversed daala_fdct_ii_N */
    fdct_ii(n, in, tmp);
    for (int k = 0; k < n; k++) out[k] = tmp[brev(lg, k)];
    return 0;
  case 2: /* Adst */
  case 3: /* FlipAdst: same 1-D kernel, flip is applied by the 2-D driver */
    if (n == 4) {
      fdst_vii_4(in, out);
      return 0;
    }
    if (n == 8) fdst_iv_8(in, tmp);
    else if (n == 16) fdst_iv_16(in, tmp);
    else return -1;
    for (int k = 0; k < n; k++) out[k] = tmp[brev(lg, k)];
    return 0;
  }
  return -1;
}

/* FWD_SHIFT_* (forward.rs:22-40), indexed [TxSize][shift_idx][stage]. */
static const int8_t FWD_SHIFT[19][3][3] = {
    {{3, 0, 0}, {2, 0, 1}, {0, 0, 3}},    /* 4x4 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 8x8 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 16x16 */
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},   /* 32x32 */
    {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}}, /* 64x64 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 4x8 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 8x4 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 8x16 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 16x8 */
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},   /* 16x32 */
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},   /* 32x16 */
    {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}}, /* 32x64 */
    {{4, -1, -2}, {2, 0, -1}, {0, 0, 1}}, /* 64x32 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 4x16 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 16x4 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 8x32 */
    {{4, -1, 0}, {2, 0, 1}, {0, 0, 3}},   /* 32x8 */
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},   /* 16x64 */
    {{4, -2, 0}, {2, 0, 0}, {0, 0, 2}},   /* 64x16 */
};

/* round_shift_array (src/transform/mod.rs:499-521): bit > 0 rounds right,
 * bit < 0 shifts left. */
static inline T rsa(T v, int bit) {
  if (bit > 0) return round_shift(v, bit);
  if (bit < 0) return (T)((uint32_t)v << -bit);
  return v;
}

/* FwdTxfm2D::fht, forward.rs:1804-1899.  The row-flipped branch
 * (:1858-1862) is unreachable in the reference (RAV1E_TX_TYPES,
 * mod.rs:34-50) and reads uninitialised lanes; row FlipAdst is rejected. */
int orc_fwd_txfm2d(const int16_t *residual, int32_t *coeffs, int tx_size,
                   int tx_type, int bit_depth) {
  if (tx_size < 0 || tx_size > 18 || tx_type < 0 || tx_type > 15) return -1;
  if (bit_depth != 8 && bit_depth != 10 && bit_depth != 12) return -1;
  int w = 1 << ORC_TX_W_LOG2[tx_size], h = 1 << ORC_TX_H_LOG2[tx_size];
  int ck = ORC_TX_COL[tx_type], rk = ORC_TX_ROW[tx_type];
  if (rk == 3) return -1;
  int si = (bit_depth - 8) / 2;
  const int8_t *sh = FWD_SHIFT[tx_size][si];
  static const T zero[64];
  T probe[64];
  /* validate both 1-D kernels exist before writing anything */
  if (orc_fwd_txfm1d(ck, h, zero, probe) || orc_fwd_txfm1d(rk, w, zero, probe))
    return -1;
  T buf[64 * 64];
  T col_in[64], col_out[64];
  for (int c = 0; c < w; c++) {
    for (int r = 0; r < h; r++) {
      int rr = ck == 3 ? h - 1 - r : r; /* Col::FLIPPED: flip upside down */
      col_in[r] = rsa((T)residual[rr * w + c], -sh[0]);
    }
    orc_fwd_txfm1d(ck, h, col_in, col_out);
    for (int r = 0; r < h; r++) buf[r * w + c] = rsa(col_out[r], -sh[1]);
  }
  for (int r = 0; r < h; r++) {
    orc_fwd_txfm1d(rk, w, buf + r * w, coeffs + r * w);
    for (int c = 0; c < w; c++)
      coeffs[r * w + c] = rsa(coeffs[r * w + c], -sh[2]);
  }
  return 0;
}

/* diff, src/encoder.rs:1044-1058 */
void orc_diff(int16_t *dst, const void *a, ptrdiff_t sa, const void *b,
              ptrdiff_t sb, int w, int h, int hbd) {
  for (int r = 0; r < h; r++)
    for (int c = 0; c < w; c++)
      dst[r * w + c] = (int16_t)((int16_t)orc_px(a, hbd, r * sa + c) -
                                 (int16_t)orc_px(b, hbd, r * sb + c));
}
