// rv_tx.h -- 1-D transform kernels for the gfx950 transform launches.
//
// Forward: the Daala integer-lifting DCT-II / DST-IV / DST-VII of
// src/transform/forward.rs:100-1700 (TxOperations :100-324, kernels
// :338-1700, 1-D dispatch txfm_types :1702-1769).  Inverse: the AV1
// normative butterflies of src/transform/inverse.rs:35-1544, written as the
// specification's stage program (AV1 spec 7.13.2) with the reference's
// per-add clamp (clamp_value, src/transform/mod.rs:490).
//
// Every kernel is a template on the point count and works on a
// register-resident array: after unrolling, every index is a compile-time
// constant, so one lane transforms one row / column entirely in VGPRs.
// All i32 arithmetic wraps (Rust release semantics).
#pragma once

#include "rv_device.h"

namespace rv {
namespace tx {

typedef int32_t T;
struct P2 {  // the reference's (half, full) lane tuples
  T h, f;
};
struct TT {
  T a, b;
};

#define RV_DI __device__ __forceinline__

// ---- TxOperations for i32 (forward.rs:114-130) ----------------------------
RV_DI T txmul(T x, int m, int s) { return wadd(wmul24(x, m), (1 << s) >> 1) >> s; }
RV_DI T rsh1(T x) { return wadd(x, x < 0 ? 1 : 0) >> 1; }
RV_DI T add_avg(T a, T b) { return wadd(a, b) >> 1; }
RV_DI T sub_avg(T a, T b) { return wsub(a, b) >> 1; }

// RotateKernelPi4 (forward.rs:164-199): kind 0 Add, 1 AddAvg, 2 Sub, 3 SubAvg
template <int K>
RV_DI TT rot_pi4(T p0, T p1, int m0, int s0, int m1, int s1) {
  T t;
  if (K == 0) t = wadd(p1, p0);
  else if (K == 1) t = add_avg(p1, p0);
  else if (K == 2) t = wsub(p1, p0);
  else t = sub_avg(p1, p0);
  T a = txmul(p0, m0, s0);
  T o0 = txmul(t, m1, s1);
  T o1 = K < 2 ? wsub(a, o0) : wadd(a, o0);
  return TT{o0, o1};
}

// RotateKernel::half_kernel (forward.rs:201-277)
enum { RADD, RADDAVG, RADDSHIFT, RSUB, RSUBAVG, RSUBSHIFT };
template <int K>
RV_DI TT rot_half(P2 p0, T p1, int m0, int s0, int m1, int s1, int m2,
                  int s2) {
  T t;
  if (K == RADD || K == RADDSHIFT) t = wadd(p1, p0.h);
  else if (K == RADDAVG) t = add_avg(p1, p0.h);
  else if (K == RSUB || K == RSUBSHIFT) t = wsub(p1, p0.h);
  else t = sub_avg(p1, p0.h);
  T a = txmul(p0.f, m0, s0), b = txmul(p1, m1, s1), c = txmul(t, m2, s2);
  T o0 = wadd(b, c);
  T sh = (K == RADDSHIFT || K == RSUBSHIFT) ? rsh1(c) : c;
  T o1 = K <= RADDSHIFT ? wsub(a, sh) : wadd(a, sh);
  return TT{o0, o1};
}
template <int K>
RV_DI TT rot(T p0, T p1, int m0, int s0, int m1, int s1, int m2, int s2) {
  return rot_half<K>(P2{p0, p0}, p1, m0, s0, m1, s1, m2, s2);
}
// RotateKernelNeg (forward.rs:222-285): AVG 0 RotateNeg, 1 RotateNegAvg
template <int AVG>
RV_DI TT rot_neg(T p0, T p1, int m0, int s0, int m1, int s1, int m2, int s2) {
  T t = AVG ? sub_avg(p0, p1) : wsub(p0, p1);
  T a = txmul(p0, m0, s0), b = txmul(p1, m1, s1), c = txmul(t, m2, s2);
  return TT{wsub(b, c), wsub(c, a)};
}

// Butterflies (forward.rs:287-324)
RV_DI void bf_add(T p0, T p1, P2 &o0, T &o1h) {
  T s = wadd(p0, p1), sh = rsh1(s);
  o0 = P2{sh, s};
  o1h = wsub(p1, sh);
}
RV_DI void bf_sub(T p0, T p1, P2 &o0, T &o1h) {
  T s = wsub(p0, p1), sh = rsh1(s);
  o0 = P2{sh, s};
  o1h = wadd(p1, sh);
}
RV_DI void bf_neg(T p0, T p1, T &o0h, P2 &o1) {
  T d = wsub(p0, p1), dh = rsh1(d);
  o0h = wsub(p0, dh);
  o1 = P2{dh, d};
}
RV_DI TT bf_add_asym(P2 p0, T p1h) {
  T p1 = wadd(p1h, p0.h);
  return TT{wsub(p0.f, p1), p1};
}
RV_DI TT bf_sub_asym(P2 p0, T p1h) {
  T p1 = wsub(p1h, p0.h);
  return TT{wadd(p0.f, p1), p1};
}
RV_DI TT bf_neg_asym(T p0h, P2 p1) {
  T p0 = wadd(p0h, p1.h);
  return TT{p0, wsub(p0, p1.f)};
}
RV_DI P2 hp(T x) { return P2{rsh1(x), x}; }

#define RV_SET(x, y, expr) \
  do {                     \
    TT r_ = (expr);        \
    x = r_.a;              \
    y = r_.b;              \
  } while (0)

// ---- 2- and 4-point kernels ----------------------------------------------
// daala_fdct_ii_2 (forward.rs:407-412)
RV_DI TT fdct_ii_2(T p0, T p1) {
  TT r = rot_pi4<3>(p1, p0, 11585, 13, 11585, 13);
  return TT{r.b, r.a};
}
// daala_fdst_iv_2 (forward.rs:414-419)
RV_DI TT fdst_iv_2(T p0, T p1) {
  return rot<RADDAVG>(p0, p1, 10703, 13, 8867, 14, 3135, 12);
}
// daala_fdst_iv_2_asym (forward.rs:342-347)
RV_DI TT fdst_iv_2_asym(P2 p0, T p1h) {
  return rot_half<RADD>(p0, p1h, 473, 9, 3135, 12, 4433, 13);
}

// daala_fdst_iv_4 (forward.rs:590-615)
RV_DI void fdst_iv_4(const T *in, T *out) {
  T q0 = in[0], q1 = in[1], q2 = in[2], q3 = in[3];
  RV_SET(q0, q3, rot<RADDSHIFT>(q0, q3, 13623, 14, 4551, 12, 565, 11));
  RV_SET(q2, q1, rot<RSUBSHIFT>(q2, q1, 16069, 14, 12785, 15, 1609, 11));
  RV_SET(q2, q3, bf_sub_asym(hp(q2), q3));
  RV_SET(q0, q1, bf_sub_asym(hp(q0), q1));
  RV_SET(q2, q1, rot_pi4<1>(q2, q1, 11585, 13, 11585, 13));
  out[0] = q0; out[1] = q1; out[2] = q2; out[3] = q3;
}
// daala_fdst_iv_4_asym (forward.rs:435-466)
RV_DI void fdst_iv_4_asym(const P2 *pp, const T *hh, T *out) {
  T q0, q1, q2, q3;
  RV_SET(q0, q3, rot_half<RADDSHIFT>(pp[0], hh[3], 9633, 14, 12873, 13, 12785, 15));
  RV_SET(q2, q1, rot_half<RSUBSHIFT>(pp[2], hh[1], 11363, 14, 18081, 15, 4551, 12));
  RV_SET(q2, q3, bf_sub_asym(hp(q2), q3));
  RV_SET(q0, q1, bf_sub_asym(hp(q0), q1));
  RV_SET(q2, q1, rot_pi4<1>(q2, q1, 11585, 13, 11585, 13));
  out[0] = q0; out[1] = q1; out[2] = q2; out[3] = q3;
}

// ---- 8-point DST-IV ------------------------------------------------------
// shared body of daala_fdst_iv_8 (forward.rs:509-562) and
// daala_fdst_iv_8_asym (forward.rs:633-687) after their first stage
template <bool ASYM>
RV_DI void fdst8_tail(T r0, T r1, T r2, T r3, T r4, T r5, T r6, T r7, T *out) {
  P2 R0, R2, R5, R7;
  T r3h, r1h, r6h, r4h;
  bf_add(r0, r3, R0, r3h);
  bf_sub(r2, r1, R2, r1h);
  bf_add(r5, r6, R5, r6h);
  bf_sub(r7, r4, R7, r4h);
  RV_SET(r7, r6, bf_add_asym(R7, r6h));
  RV_SET(r5, r3, bf_add_asym(R5, r3h));
  RV_SET(r2, r4, bf_add_asym(R2, r4h));
  RV_SET(r0, r1, bf_sub_asym(R0, r1h));
  if (!ASYM) {
    RV_SET(r3, r4, rot<RSUBAVG>(r3, r4, 10703, 13, 8867, 14, 3135, 12));
    RV_SET(r2, r5, rot_neg<1>(r2, r5, 10703, 13, 8867, 14, 3135, 12));
    RV_SET(r1, r6, rot_pi4<3>(r1, r6, 11585, 13, 11585, 13));
  } else {
    RV_SET(r3, r4, rot<RSUBAVG>(r3, r4, 669, 9, 8867, 14, 3135, 12));
    RV_SET(r2, r5, rot_neg<1>(r2, r5, 669, 9, 8867, 14, 3135, 12));
    RV_SET(r1, r6, rot_pi4<3>(r1, r6, 5793, 12, 11585, 13));
  }
  out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3;
  out[4] = r4; out[5] = r5; out[6] = r6; out[7] = r7;
}
RV_DI void fdst_iv_8(const T *in, T *out) {
  T r0 = in[0], r1 = in[1], r2 = in[2], r3 = in[3], r4 = in[4], r5 = in[5],
    r6 = in[6], r7 = in[7];
  RV_SET(r0, r7, rot<RADD>(r0, r7, 17911, 14, 14699, 14, 803, 13));
  RV_SET(r6, r1, rot<RSUB>(r6, r1, 20435, 14, 21845, 15, 1189, 12));
  RV_SET(r2, r5, rot<RADD>(r2, r5, 22173, 14, 3363, 13, 15447, 15));
  RV_SET(r4, r3, rot<RSUB>(r4, r3, 23059, 14, 2271, 14, 5197, 13));
  fdst8_tail<false>(r0, r1, r2, r3, r4, r5, r6, r7, out);
}
RV_DI void fdst_iv_8_asym(const P2 *pp, const T *hh, T *out) {
  T r0, r1, r2, r3, r4, r5, r6, r7;
  RV_SET(r0, r7, rot_half<RADD>(pp[0], hh[7], 12665, 14, 5197, 12, 2271, 14));
  RV_SET(r6, r1, rot_half<RSUB>(pp[6], hh[1], 14449, 14, 30893, 15, 3363, 13));
  RV_SET(r2, r5, rot_half<RADD>(pp[2], hh[5], 15679, 14, 1189, 11, 5461, 13));
  RV_SET(r4, r3, rot_half<RSUB>(pp[4], hh[3], 16305, 14, 803, 12, 14699, 14));
  fdst8_tail<true>(r0, r1, r2, r3, r4, r5, r6, r7, out);
}

// ---- 16-point DST-IV -----------------------------------------------------
// Stages 1, 2, 4, 5 of daala_fdst_iv_16 (forward.rs:797-868) and
// daala_fdst_iv_16_asym (forward.rs:994-1065); stage 3 and 5 differ.
template <bool ASYM>
RV_DI void fdst16_core(T *s) {
  P2 S0, S2, Sd, Sf, Pt;
  T s3h, seh, s1h, sch, s4h, sbh, s6h, s9h;
  RV_SET(s[0], s[7], bf_sub_asym(hp(s[0]), s[7]));
  RV_SET(s[8], s[15], bf_sub_asym(hp(s[8]), s[15]));
  RV_SET(s[4], s[3], bf_add_asym(hp(s[4]), s[3]));
  RV_SET(s[12], s[11], bf_add_asym(hp(s[12]), s[11]));
  RV_SET(s[2], s[5], bf_sub_asym(hp(s[2]), s[5]));
  RV_SET(s[10], s[13], bf_sub_asym(hp(s[10]), s[13]));
  RV_SET(s[6], s[1], bf_add_asym(hp(s[6]), s[1]));
  RV_SET(s[14], s[9], bf_add_asym(hp(s[14]), s[9]));
  bf_add(s[8], s[4], Pt, s4h);
  s[8] = Pt.f;
  bf_add(s[7], s[11], Pt, sbh);
  s[7] = Pt.f;
  bf_sub(s[10], s[6], Pt, s6h);
  s[10] = Pt.f;
  bf_sub(s[5], s[9], Pt, s9h);
  s[5] = Pt.f;
  bf_add(s[0], s[3], S0, s3h);
  bf_add(s[13], s[14], Sd, seh);
  bf_sub(s[2], s[1], S2, s1h);
  bf_sub(s[15], s[12], Sf, sch);
  if (!ASYM) {  // forward.rs:818-837
    RV_SET(s[8], s[7], rot<RADDAVG>(s[8], s[7], 301, 8, 1609, 11, 12785, 15));
    RV_SET(s[9], s[6], rot<RADD>(s9h, s6h, 11363, 13, 9041, 15, 4551, 13));
    RV_SET(s[5], s[10], rot_neg<1>(s[5], s[10], 5681, 12, 9041, 15, 4551, 12));
    RV_SET(s[4], s[11], rot_neg<0>(s4h, sbh, 9633, 13, 12873, 14, 6393, 15));
  } else {  // forward.rs:1015-1034
    RV_SET(s[8], s[7], rot<RADD>(s[8], s[7], 9633, 13, 12873, 14, 6393, 15));
    RV_SET(s[9], s[6], rot<RADD>(s9h, s6h, 22725, 14, 9041, 15, 4551, 13));
    RV_SET(s[5], s[10], rot_neg<0>(s[5], s[10], 11363, 13, 9041, 15, 4551, 13));
    RV_SET(s[4], s[11], rot_neg<0>(s4h, sbh, 9633, 13, 12873, 14, 6393, 15));
  }
  RV_SET(s[2], s[12], bf_add_asym(S2, sch));
  RV_SET(s[0], s[1], bf_sub_asym(S0, s1h));
  RV_SET(s[15], s[14], bf_add_asym(Sf, seh));
  RV_SET(s[13], s[3], bf_add_asym(Sd, s3h));
  RV_SET(s[7], s[6], bf_add_asym(hp(s[7]), s[6]));
  RV_SET(s[8], s[9], bf_sub_asym(hp(s[8]), s[9]));
  RV_SET(s[10], s[11], bf_sub_asym(hp(s[10]), s[11]));
  RV_SET(s[5], s[4], bf_add_asym(hp(s[5]), s[4]));
  if (!ASYM) {  // forward.rs:850-868
    RV_SET(s[12], s[3], rot<RADDAVG>(s[12], s[3], 669, 9, 8867, 14, 3135, 12));
    RV_SET(s[2], s[13], rot_neg<1>(s[2], s[13], 669, 9, 8867, 14, 3135, 12));
    RV_SET(s[10], s[5], rot_pi4<1>(s[10], s[5], 5793, 12, 11585, 13));
    RV_SET(s[6], s[9], rot_pi4<1>(s[6], s[9], 5793, 12, 11585, 13));
    RV_SET(s[14], s[1], rot_pi4<1>(s[14], s[1], 5793, 12, 11585, 13));
  } else {  // forward.rs:1047-1065
    RV_SET(s[12], s[3], rot<RADD>(s[12], s[3], 10703, 13, 8867, 14, 3135, 13));
    RV_SET(s[2], s[13], rot_neg<0>(s[2], s[13], 10703, 13, 8867, 14, 3135, 13));
    RV_SET(s[10], s[5], rot_pi4<0>(s[10], s[5], 11585, 13, 5793, 13));
    RV_SET(s[6], s[9], rot_pi4<0>(s[6], s[9], 11585, 13, 5793, 13));
    RV_SET(s[14], s[1], rot_pi4<0>(s[14], s[1], 11585, 13, 5793, 13));
  }
}
// daala_fdst_iv_16 (forward.rs:751-873)
RV_DI void fdst_iv_16(const T *in, T *out) {
  T s[16];
#pragma unroll
  for (int i = 0; i < 16; i++) s[i] = in[i];
  RV_SET(s[0], s[15], rot<RADDSHIFT>(s[0], s[15], 24279, 15, 11003, 13, 1137, 14));
  RV_SET(s[14], s[1], rot<RSUBSHIFT>(s[14], s[1], 1645, 11, 305, 8, 425, 11));
  RV_SET(s[2], s[13], rot<RADDSHIFT>(s[2], s[13], 14053, 14, 8423, 13, 2815, 13));
  RV_SET(s[12], s[3], rot<RSUBSHIFT>(s[12], s[3], 14811, 14, 7005, 13, 3903, 13));
  RV_SET(s[4], s[11], rot<RADDSHIFT>(s[4], s[11], 30853, 15, 11039, 14, 9907, 14));
  RV_SET(s[10], s[5], rot<RSUBSHIFT>(s[10], s[5], 15893, 14, 3981, 13, 1489, 11));
  RV_SET(s[6], s[9], rot<RADDSHIFT>(s[6], s[9], 32413, 15, 601, 11, 13803, 14));
  RV_SET(s[8], s[7], rot<RSUBSHIFT>(s[8], s[7], 32729, 15, 201, 11, 1945, 11));
  fdst16_core<false>(s);
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = s[i];
}
// daala_fdst_iv_16_asym (forward.rs:938-1070)
RV_DI void fdst_iv_16_asym(const P2 *pp, const T *hh, T *out) {
  T s[16];
  RV_SET(s[0], s[15], rot_half<RADDSHIFT>(pp[0], hh[15], 1073, 11, 62241, 15, 201, 11));
  RV_SET(s[14], s[1], rot_half<RSUBSHIFT>(pp[14], hh[1], 18611, 15, 55211, 15, 601, 11));
  RV_SET(s[2], s[13], rot_half<RADDSHIFT>(pp[2], hh[13], 9937, 14, 1489, 10, 3981, 13));
  RV_SET(s[12], s[3], rot_half<RSUBSHIFT>(pp[12], hh[3], 10473, 14, 39627, 15, 11039, 14));
  RV_SET(s[4], s[11], rot_half<RADDSHIFT>(pp[4], hh[11], 2727, 12, 3903, 12, 7005, 13));
  RV_SET(s[10], s[5], rot_half<RSUBSHIFT>(pp[10], hh[5], 5619, 13, 2815, 12, 8423, 13));
  // the reference's constant is 13599 (its comment says 13588), forward.rs:984
  RV_SET(s[6], s[9], rot_half<RADDSHIFT>(pp[6], hh[9], 2865, 12, 13599, 15, 305, 8));
  RV_SET(s[8], s[7], rot_half<RSUBSHIFT>(pp[8], hh[7], 23143, 15, 1137, 13, 11003, 13));
  fdst16_core<true>(s);
#pragma unroll
  for (int i = 0; i < 16; i++) out[i] = s[i];
}

// ---- 32-point DST-IV (asymmetric input), forward.rs:1279-1548 -------------
RV_DI void fdst_iv_32_asym(const P2 *pp, const T *hh, T *t) {
  RV_SET(t[0], t[31], rot_half<RADD>(pp[0], hh[31], 5933, 13, 22595, 14, 1137, 15));
  RV_SET(t[30], t[1], rot_half<RSUB>(pp[30], hh[1], 6203, 13, 21403, 14, 3409, 15));
  RV_SET(t[2], t[29], rot_half<RADD>(pp[2], hh[29], 25833, 15, 315, 8, 5673, 15));
  RV_SET(t[28], t[3], rot_half<RSUB>(pp[28], hh[3], 26791, 15, 4717, 12, 7923, 15));
  RV_SET(t[4], t[27], rot_half<RADD>(pp[4], hh[27], 6921, 13, 17531, 14, 10153, 15));
  RV_SET(t[26], t[5], rot_half<RSUB>(pp[26], hh[5], 28511, 15, 32303, 15, 1545, 12));
  RV_SET(t[6], t[25], rot_half<RADD>(pp[6], hh[25], 29269, 15, 14733, 14, 1817, 12));
  RV_SET(t[24], t[7], rot_half<RSUB>(pp[24], hh[7], 29957, 15, 13279, 14, 8339, 14));
  RV_SET(t[8], t[23], rot_half<RADD>(pp[8], hh[23], 7643, 13, 11793, 14, 18779, 15));
  RV_SET(t[22], t[9], rot_half<RSUB>(pp[22], hh[9], 15557, 14, 20557, 15, 20835, 15));
  RV_SET(t[10], t[21], rot_half<RADD>(pp[10], hh[21], 31581, 15, 17479, 15, 22841, 15));
  RV_SET(t[20], t[11], rot_half<RSUB>(pp[20], hh[11], 7993, 13, 14359, 15, 3099, 12));
  RV_SET(t[12], t[19], rot_half<RADD>(pp[12], hh[19], 16143, 14, 2801, 13, 26683, 15));
  RV_SET(t[18], t[13], rot_half<RSUB>(pp[18], hh[13], 16261, 14, 4011, 14, 14255, 14));
  RV_SET(t[14], t[17], rot_half<RADD>(pp[14], hh[17], 32679, 15, 4821, 15, 30269, 15));
  RV_SET(t[16], t[15], rot_half<RSUB>(pp[16], hh[15], 16379, 14, 201, 12, 15977, 14));

  P2 P[32];
  T H[32];
  bf_add(t[0], t[15], P[0], H[15]);
  bf_sub(t[31], t[16], P[31], H[16]);
  bf_add(t[17], t[30], P[17], H[30]);
  bf_sub(t[14], t[1], P[14], H[1]);
  bf_add(t[2], t[13], P[2], H[13]);
  bf_sub(t[29], t[18], P[29], H[18]);
  bf_add(t[19], t[28], P[19], H[28]);
  bf_sub(t[12], t[3], P[12], H[3]);
  bf_add(t[4], t[11], P[4], H[11]);
  bf_sub(t[27], t[20], P[27], H[20]);
  bf_add(t[21], t[26], P[21], H[26]);
  bf_sub(t[10], t[5], P[10], H[5]);
  bf_add(t[6], t[9], P[6], H[9]);
  bf_sub(t[25], t[22], P[25], H[22]);
  bf_add(t[23], t[24], P[23], H[24]);
  bf_sub(t[8], t[7], P[8], H[7]);

  RV_SET(t[0], t[7], bf_sub_asym(P[0], H[7]));
  RV_SET(t[31], t[24], bf_add_asym(P[31], H[24]));
  RV_SET(t[25], t[30], bf_sub_asym(P[25], H[30]));
  RV_SET(t[6], t[1], bf_add_asym(P[6], H[1]));
  RV_SET(t[2], t[5], bf_sub_asym(P[2], H[5]));
  RV_SET(t[29], t[26], bf_add_asym(P[29], H[26]));
  RV_SET(t[27], t[28], bf_sub_asym(P[27], H[28]));
  RV_SET(t[4], t[3], bf_add_asym(P[4], H[3]));
  RV_SET(t[8], t[16], bf_add_asym(P[8], H[16]));
  RV_SET(t[14], t[22], bf_sub_asym(P[14], H[22]));
  RV_SET(t[23], t[15], bf_add_asym(P[23], H[15]));
  RV_SET(t[17], t[9], bf_sub_asym(P[17], H[9]));
  RV_SET(t[10], t[18], bf_add_asym(P[10], H[18]));
  RV_SET(t[12], t[20], bf_sub_asym(P[12], H[20]));
  RV_SET(t[21], t[13], bf_add_asym(P[21], H[13]));
  RV_SET(t[19], t[11], bf_sub_asym(P[19], H[11]));

  RV_SET(t[15], t[16], rot<RSUB>(t[15], t[16], 17911, 14, 14699, 14, 803, 13));
  RV_SET(t[17], t[14], rot<RADD>(t[17], t[14], 10217, 13, 5461, 13, 1189, 12));
  RV_SET(t[18], t[13], rot<RADD>(t[18], t[13], 5543, 12, 3363, 13, 7723, 14));
  RV_SET(t[12], t[19], rot<RSUB>(t[12], t[19], 11529, 13, 2271, 14, 5197, 13));
  RV_SET(t[11], t[20], rot_neg<0>(t[11], t[20], 11529, 13, 2271, 14, 5197, 13));
  RV_SET(t[10], t[21], rot_neg<0>(t[10], t[21], 5543, 12, 3363, 13, 7723, 14));
  RV_SET(t[9], t[22], rot_neg<0>(t[9], t[22], 10217, 13, 5461, 13, 1189, 12));
  RV_SET(t[8], t[23], rot_neg<0>(t[8], t[23], 17911, 14, 14699, 14, 803, 13));

  P2 Q[32];
  T G[32];
  bf_sub(t[3], t[0], Q[3], G[0]);
  bf_add(t[28], t[31], Q[28], G[31]);
  bf_sub(t[30], t[29], Q[30], G[29]);
  bf_add(t[1], t[2], Q[1], G[2]);
  bf_add(t[24], t[4], Q[24], G[4]);
  bf_sub(t[26], t[6], Q[26], G[6]);
  bf_add(t[7], t[27], Q[7], G[27]);
  bf_sub(t[5], t[25], Q[5], G[25]);
  bf_sub(t[11], t[8], Q[11], G[8]);
  bf_add(t[20], t[23], Q[20], G[23]);
  bf_sub(t[22], t[21], Q[22], G[21]);
  bf_add(t[9], t[10], Q[9], G[10]);
  bf_sub(t[15], t[12], Q[15], G[12]);
  bf_add(t[16], t[19], Q[16], G[19]);
  bf_sub(t[18], t[17], Q[18], G[17]);
  bf_add(t[13], t[14], Q[13], G[14]);
  t[24] = Q[24].f;
  t[26] = Q[26].f;
  t[7] = Q[7].f;
  t[5] = Q[5].f;

  RV_SET(t[24], t[7], rot<RADD>(t[24], t[7], 301, 8, 1609, 11, 6393, 15));
  RV_SET(G[25], G[6], rot<RADD>(G[25], G[6], 11363, 13, 9041, 15, 4551, 13));
  RV_SET(t[5], t[26], rot_neg<0>(t[5], t[26], 5681, 12, 9041, 15, 4551, 13));
  RV_SET(G[4], G[27], rot_neg<0>(G[4], G[27], 9633, 13, 12873, 14, 6393, 15));

  RV_SET(t[1], t[0], bf_add_asym(Q[1], G[0]));
  RV_SET(t[30], t[31], bf_sub_asym(Q[30], G[31]));
  RV_SET(t[28], t[2], bf_sub_asym(Q[28], G[2]));
  RV_SET(t[3], t[29], bf_sub_asym(Q[3], G[29]));
  RV_SET(t[5], t[4], bf_add_asym(hp(t[5]), G[4]));
  RV_SET(t[26], t[27], bf_sub_asym(hp(t[26]), G[27]));
  RV_SET(t[7], t[6], bf_add_asym(hp(t[7]), G[6]));
  RV_SET(t[24], t[25], bf_sub_asym(hp(t[24]), G[25]));
  RV_SET(t[9], t[8], bf_add_asym(Q[9], G[8]));
  RV_SET(t[22], t[23], bf_sub_asym(Q[22], G[23]));
  RV_SET(t[20], t[10], bf_sub_asym(Q[20], G[10]));
  RV_SET(t[11], t[21], bf_sub_asym(Q[11], G[21]));
  RV_SET(t[18], t[12], bf_add_asym(Q[18], G[12]));
  RV_SET(t[13], t[19], bf_add_asym(Q[13], G[19]));
  RV_SET(t[15], t[14], bf_add_asym(Q[15], G[14]));
  RV_SET(t[16], t[17], bf_sub_asym(Q[16], G[17]));

  RV_SET(t[2], t[29], rot_neg<0>(t[2], t[29], 669, 9, 8867, 14, 3135, 13));
  RV_SET(t[28], t[3], rot<RADD>(t[28], t[3], 669, 9, 8867, 14, 3135, 13));
  RV_SET(t[10], t[21], rot_neg<0>(t[10], t[21], 669, 9, 8867, 14, 3135, 13));
  RV_SET(t[20], t[11], rot<RADD>(t[20], t[11], 669, 9, 8867, 14, 3135, 13));
  RV_SET(t[12], t[19], rot<RADD>(t[12], t[19], 669, 9, 8867, 14, 3135, 13));
  RV_SET(t[18], t[13], rot_neg<0>(t[18], t[13], 669, 9, 8867, 14, 3135, 13));
  RV_SET(t[30], t[1], rot_pi4<0>(t[30], t[1], 5793, 12, 5793, 13));
  RV_SET(t[26], t[5], rot_pi4<0>(t[26], t[5], 5793, 12, 5793, 13));
  RV_SET(t[25], t[6], rot_pi4<2>(t[25], t[6], 5793, 12, 5793, 13));
  RV_SET(t[22], t[9], rot_pi4<0>(t[22], t[9], 5793, 12, 5793, 13));
  RV_SET(t[14], t[17], rot_pi4<0>(t[14], t[17], 5793, 12, 5793, 13));
}

// ---- DCT-II recursion -----------------------------------------------------
template <int N>
RV_DI void fdct_ii(const T *x, T *out);

// daala_fdct_ii_N_asym, N = 4..32 (forward.rs:421-433, 617-631, 917-936,
// 1212-1277): even inputs are halves, odd inputs are pairs.
template <int N>
RV_DI void fdct_ii_asym(const T *hh, const P2 *pp, T *out) {
  constexpr int M = N / 2;
  T x[N];
#pragma unroll
  for (int i = 0; i < M; i++) {
    const int j = N - 1 - i;
    TT r = (i & 1) ? bf_sub_asym(pp[i], hh[j]) : bf_neg_asym(hh[i], pp[j]);
    x[i] = r.a;
    x[j] = r.b;
  }
  T lo[M], hi[M], rev[M];
#pragma unroll
  for (int k = 0; k < M; k++) rev[k] = x[N - 1 - k];
  if constexpr (N == 4) {
    TT a = fdct_ii_2(x[0], x[1]);
    TT b = fdst_iv_2(rev[0], rev[1]);
    lo[0] = a.a; lo[1] = a.b;
    hi[0] = b.a; hi[1] = b.b;
  } else {
    fdct_ii<M>(x, lo);
    if constexpr (M == 4) fdst_iv_4(rev, hi);
    else if constexpr (M == 8) fdst_iv_8(rev, hi);
    else fdst_iv_16(rev, hi);
  }
#pragma unroll
  for (int k = 0; k < M; k++) {
    out[k] = lo[k];
    out[M + k] = hi[M - 1 - k];
  }
}

// daala_fdct_ii_N, N = 4..64 (forward.rs:349-361, 468-481, 689-707,
// 1072-1136, 1551-1658)
template <int N>
RV_DI void fdct_ii(const T *x, T *out) {
  constexpr int M = N / 2;
  T hh[N];
  P2 pp[N];
#pragma unroll
  for (int i = 0; i < M; i++) {
    const int j = N - 1 - i;
    if (i & 1) bf_add(x[i], x[j], pp[i], hh[j]);
    else bf_neg(x[i], x[j], hh[i], pp[j]);
  }
  // the DST half receives (P[n-1], H[n-2], P[n-3], ...)
  P2 dp[M];
  T dh[M];
#pragma unroll
  for (int k = 0; k < M; k++) {
    if (k & 1) {
      dh[k] = hh[N - 1 - k];
      dp[k] = P2{0, 0};
    } else {
      dp[k] = pp[N - 1 - k];
      dh[k] = 0;
    }
  }
  T lo[M], hi[M];
  if constexpr (N == 4) {
    TT a = bf_neg_asym(hh[0], pp[1]);  // daala_fdct_ii_2_asym
    TT b = fdst_iv_2_asym(dp[0], dh[1]);
    lo[0] = a.a; lo[1] = a.b;
    hi[0] = b.a; hi[1] = b.b;
  } else {
    fdct_ii_asym<M>(hh, pp, lo);
    if constexpr (M == 4) fdst_iv_4_asym(dp, dh, hi);
    else if constexpr (M == 8) fdst_iv_8_asym(dp, dh, hi);
    else if constexpr (M == 16) fdst_iv_16_asym(dp, dh, hi);
    else fdst_iv_32_asym(dp, dh, hi);
  }
#pragma unroll
  for (int k = 0; k < M; k++) {
    out[k] = lo[k];
    out[M + k] = hi[M - 1 - k];
  }
}

template <int LG>
__host__ __device__ constexpr int brev(int x) {
  int r = 0;
  for (int i = 0; i < LG; i++) r |= ((x >> i) & 1) << (LG - 1 - i);
  return r;
}
template <int N>
__host__ __device__ constexpr int lg2() {
  return N == 4 ? 2 : N == 8 ? 3 : N == 16 ? 4 : N == 32 ? 5 : 6;
}

// daala_fdst_vii_4 (forward.rs:375-405)
RV_DI void fdst_vii_4(const T *in, T *out) {
  T q0 = in[0], q1 = in[1], q2 = in[2], q3 = in[3];
  T t0 = wadd(q1, q3);
  T t1 = wadd(q1, sub_avg(q0, t0));
  T t2 = wsub(q0, q1);
  T t3 = q2;
  T t4 = wadd(q0, q3);
  t0 = txmul(t0, 7021, 14);
  t1 = txmul(t1, 37837, 15);
  t2 = txmul(t2, 21513, 15);
  t3 = txmul(t3, 37837, 15);
  t4 = txmul(t4, 467, 11);
  T t3h = rsh1(t3);
  T u4 = wadd(t4, t3h);
  out[0] = wadd(t0, u4);
  out[1] = t1;
  out[2] = wadd(t0, wsub(t2, t3h));
  out[3] = wadd(t2, wsub(t3, u4));
}

// Kind ids in TBL_IDX order (src/transform/mod.rs:158-173):
// 0 Id, 1 Dct, 2 Adst, 3 FlipAdst.
__host__ __device__ constexpr bool fwd_supported(int kind, int n) {
  return kind == 0 ? n <= 32 : kind == 1 ? true : n <= 16;
}
__host__ __device__ constexpr bool inv_supported(int kind, int n) {
  return kind == 0 ? n <= 32 : kind == 1 ? true : kind == 2 ? n <= 16 : false;
}

// txfm_types::Detail::forward (forward.rs:1745-1768): in/out may alias.
template <int KIND, int N>
RV_DI void fwd1d(const T *in, T *out) {
  constexpr int LG = lg2<N>();
  if constexpr (KIND == 0) {
#pragma unroll
    for (int i = 0; i < N; i++) out[i] = in[i];
  } else if constexpr (KIND == 1) {
    T tmp[N];
    fdct_ii<N>(in, tmp);
#pragma unroll
    for (int k = 0; k < N; k++) out[k] = tmp[brev<LG>(k)];
  } else {
    if constexpr (N == 4) {
      T tmp[4];
      fdst_vii_4(in, tmp);
#pragma unroll
      for (int k = 0; k < 4; k++) out[k] = tmp[k];
    } else {
      T tmp[N];
      if constexpr (N == 8) fdst_iv_8(in, tmp);
      else fdst_iv_16(in, tmp);
#pragma unroll
      for (int k = 0; k < N; k++) out[k] = tmp[brev<LG>(k)];
    }
  }
}

// ---- inverse (AV1 spec 7.13.2, reference inverse.rs:35-1544) -------------
// COSPI_INV (inverse.rs:22-29) extended to the spec's cos128 / sin128.
__host__ __device__ constexpr int32_t cospi_c(int k) {
  constexpr int32_t c[65] = {
      4096, 4095, 4091, 4085, 4076, 4065, 4052, 4036, 4017, 3996, 3973,
      3948, 3920, 3889, 3857, 3822, 3784, 3745, 3703, 3659, 3612, 3564,
      3513, 3461, 3406, 3349, 3290, 3229, 3166, 3102, 3035, 2967, 2896,
      2824, 2751, 2675, 2598, 2520, 2440, 2359, 2276, 2191, 2106, 2019,
      1931, 1842, 1751, 1660, 1567, 1474, 1380, 1285, 1189, 1092, 995,
      897,  799,  700,  601,  501,  401,  301,  201,  101,  0};
  return c[k];
}
__host__ __device__ constexpr int32_t cos128(int angle) {
  const int a = angle & 255;
  return a <= 64 ? cospi_c(a)
                 : a <= 128 ? -cospi_c(128 - a)
                            : a <= 192 ? -cospi_c(a - 128) : cospi_c(256 - a);
}
__host__ __device__ constexpr int32_t sin128(int angle) {
  return cos128(angle - 64);
}

// clamp_value (src/transform/mod.rs:490) for bit <= 31: one v_med3_i32
RV_DI T clampv(T v, int bit) {
  const T hi = (T)((1u << (bit - 1)) - 1u), lo = -hi - 1;
  return __builtin_elementwise_min(__builtin_elementwise_max(v, lo), hi);
}
// half_btf (src/transform/mod.rs:476-488)
RV_DI T half_btf(T w0, T in0, T w1, T in1) {
  return wadd(wadd(wmul24(w0, in0), wmul24(w1, in1)), 1 << 11) >> 12;
}
// B(a, b, angle, flip) and H(a, b, flip) of the spec's butterfly program.
RV_DI void Bf(T *t, int a, int b, int angle, int flip) {
  const T c = cos128(angle), s = sin128(angle);
  const T x = half_btf(c, t[a], -s, t[b]);
  const T y = half_btf(s, t[a], c, t[b]);
  if (flip) {
    t[a] = y;
    t[b] = x;
  } else {
    t[a] = x;
    t[b] = y;
  }
}
RV_DI void Hf(T *t, int a, int b, int flip, int r) {
  if (flip) {
    const int tmp = a;
    a = b;
    b = tmp;
  }
  const T x = t[a], y = t[b];
  t[a] = clampv(wadd(x, y), r);
  t[b] = clampv(wsub(x, y), r);
}

// Inverse DCT process (spec 7.13.2.3), 2^n points.
template <int n>
RV_DI void idct(T *t, int r) {
  constexpr int n0 = 1 << n;
  {
    T c[n0];
#pragma unroll
    for (int i = 0; i < n0; i++) c[i] = t[i];
#pragma unroll
    for (int i = 0; i < n0; i++) t[i] = c[brev<n>(i)];
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 16; i++) Bf(t, 32 + i, 63 - i, 63 - 4 * brev<4>(i), 0);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 8; i++) Bf(t, 16 + i, 31 - i, 6 + (brev<3>(7 - i) << 3), 0);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 16; i++) Hf(t, 32 + i * 2, 33 + i * 2, i & 1, r);
  }
  if constexpr (n >= 4) {
#pragma unroll
    for (int i = 0; i < 4; i++) Bf(t, 8 + i, 15 - i, 12 + (brev<2>(3 - i) << 4), 0);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 8; i++) Hf(t, 16 + 2 * i, 17 + 2 * i, i & 1, r);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 2; j++)
        Bf(t, 62 - i * 4 - j, 33 + i * 4 + j, 60 - 16 * brev<2>(i) + 64 * j, 1);
  }
  if constexpr (n >= 3) {
#pragma unroll
    for (int i = 0; i < 2; i++) Bf(t, 4 + i, 7 - i, 56 - 32 * i, 0);
  }
  if constexpr (n >= 4) {
#pragma unroll
    for (int i = 0; i < 4; i++) Hf(t, 8 + 2 * i, 9 + 2 * i, i & 1, r);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++)
        Bf(t, 30 - 4 * i - j, 17 + 4 * i + j, 24 + (j << 6) + ((1 - i) << 5), 1);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 8; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) Hf(t, 32 + i * 4 + j, 35 + i * 4 - j, i & 1, r);
  }
#pragma unroll
  for (int i = 0; i < 2; i++) Bf(t, 2 * i, 2 * i + 1, 32 + 16 * i, 1 - i);
  if constexpr (n >= 3) {
#pragma unroll
    for (int i = 0; i < 2; i++) Hf(t, 4 + 2 * i, 5 + 2 * i, i, r);
  }
  if constexpr (n >= 4) {
#pragma unroll
    for (int i = 0; i < 2; i++) Bf(t, 14 - i, 9 + i, 48 + 64 * i, 1);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) Hf(t, 16 + 4 * i + j, 19 + 4 * i - j, i & 1, r);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 4; j++)
        Bf(t, 61 - i * 8 - j, 34 + i * 8 + j, 56 - i * 32 + (j >> 1) * 64, 1);
  }
#pragma unroll
  for (int i = 0; i < 2; i++) Hf(t, i, 3 - i, 0, r);
  if constexpr (n >= 3) Bf(t, 6, 5, 32, 1);
  if constexpr (n >= 4) {
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 2; j++) Hf(t, 8 + 4 * i + j, 11 + 4 * i - j, i, r);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 4; i++) Bf(t, 29 - i, 18 + i, 48 + (i >> 1) * 64, 1);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) Hf(t, 32 + 8 * i + j, 39 + 8 * i - j, i & 1, r);
  }
  if constexpr (n >= 3) {
#pragma unroll
    for (int i = 0; i < 4; i++) Hf(t, i, 7 - i, 0, r);
  }
  if constexpr (n >= 4) {
#pragma unroll
    for (int i = 0; i < 2; i++) Bf(t, 13 - i, 10 + i, 32, 1);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) Hf(t, 16 + i * 8 + j, 23 + i * 8 - j, i, r);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 8; i++) Bf(t, 59 - i, 36 + i, i < 4 ? 48 : 112, 1);
  }
  if constexpr (n >= 4) {
#pragma unroll
    for (int i = 0; i < 8; i++) Hf(t, i, 15 - i, 0, r);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 4; i++) Bf(t, 27 - i, 20 + i, 32, 1);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 8; i++) Hf(t, 32 + i, 47 - i, 0, r);
#pragma unroll
    for (int i = 0; i < 8; i++) Hf(t, 48 + i, 63 - i, 1, r);
  }
  if constexpr (n >= 5) {
#pragma unroll
    for (int i = 0; i < 16; i++) Hf(t, i, 31 - i, 0, r);
  }
  if constexpr (n == 6) {
#pragma unroll
    for (int i = 0; i < 8; i++) Bf(t, 55 - i, 40 + i, 32, 1);
#pragma unroll
    for (int i = 0; i < 32; i++) Hf(t, i, 63 - i, 0, r);
  }
}

// av1_iadst4 (inverse.rs:63-109): SINPI_INV (inverse.rs:31), no clamps
RV_DI void iadst4(T *t) {
  const T x0 = t[0], x1 = t[1], x2 = t[2], x3 = t[3];
  T s0 = wmul24(1321, x0), s1 = wmul24(2482, x0);
  T s2 = wmul24(3344, x1), s3 = wmul24(3803, x2);
  T s4 = wmul24(1321, x2), s5 = wmul24(2482, x3);
  T s6 = wmul24(3803, x3);
  T s7 = wadd(wsub(x0, x2), x3);
  s0 = wadd(s0, s3);
  s1 = wsub(s1, s4);
  s3 = s2;
  s2 = wmul24(3344, s7);
  s0 = wadd(s0, s5);
  s1 = wsub(s1, s6);
  const T y0 = wadd(s0, s3), y1 = wadd(s1, s3), y2 = s2;
  const T y3 = wsub(wadd(s0, s1), s3);
  t[0] = round_shift(y0, 12);
  t[1] = round_shift(y1, 12);
  t[2] = round_shift(y2, 12);
  t[3] = round_shift(y3, 12);
}

// ADST input / output permutations (spec 7.13.2.7 / 7.13.2.8)
template <int n>
RV_DI void adst_in_perm(T *t) {
  constexpr int n0 = 1 << n;
  T c[n0];
#pragma unroll
  for (int i = 0; i < n0; i++) c[i] = t[i];
#pragma unroll
  for (int i = 0; i < n0; i++) t[i] = c[(i & 1) ? (i - 1) : (n0 - i - 1)];
}
template <int n>
__host__ __device__ constexpr int adst_out_idx(int i) {
  return ((((i & 1) ^ ((i >> 1) & 1)) << 3) | ((((i >> 1) & 1) ^ ((i >> 2) & 1)) << 2) |
          ((((i >> 2) & 1) ^ ((i >> 3) & 1)) << 1) | ((i >> 3) & 1)) >> (4 - n);
}
template <int n>
RV_DI void adst_out_perm(T *t) {
  constexpr int n0 = 1 << n;
  T c[n0];
#pragma unroll
  for (int i = 0; i < n0; i++) c[i] = t[i];
#pragma unroll
  for (int i = 0; i < n0; i++) {
    const T v = c[adst_out_idx<n>(i)];
    t[i] = (i & 1) ? wsub(0, v) : v;
  }
}
// av1_iadst8 (inverse.rs:173-252)
RV_DI void iadst8(T *t, int r) {
  adst_in_perm<3>(t);
#pragma unroll
  for (int i = 0; i < 4; i++) Bf(t, 2 * i, 1 + 2 * i, 60 - 16 * i, 1);
#pragma unroll
  for (int i = 0; i < 4; i++) Hf(t, i, 4 + i, 0, r);
#pragma unroll
  for (int i = 0; i < 2; i++) Bf(t, 4 + 3 * i, 5 + i, 48 - 32 * i, 1);
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) Hf(t, 4 * j + i, 2 + 4 * j + i, 0, r);
#pragma unroll
  for (int i = 0; i < 2; i++) Bf(t, 2 + 4 * i, 3 + 4 * i, 32, 1);
  adst_out_perm<3>(t);
}
// av1_iadst16 (inverse.rs:364-532)
RV_DI void iadst16(T *t, int r) {
  adst_in_perm<4>(t);
#pragma unroll
  for (int i = 0; i < 8; i++) Bf(t, 2 * i, 1 + 2 * i, 62 - 8 * i, 1);
#pragma unroll
  for (int i = 0; i < 8; i++) Hf(t, i, 8 + i, 0, r);
#pragma unroll
  for (int i = 0; i < 2; i++) {
    Bf(t, 8 + 2 * i, 9 + 2 * i, 56 - 32 * i, 1);
    Bf(t, 13 + 2 * i, 12 + 2 * i, 8 + 32 * i, 1);
  }
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) Hf(t, 8 * j + i, 4 + 8 * j + i, 0, r);
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 2; j++) Bf(t, 4 + 8 * j + 3 * i, 5 + 8 * j + i, 48 - 32 * i, 1);
#pragma unroll
  for (int i = 0; i < 2; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) Hf(t, 4 * j + i, 2 + 4 * j + i, 0, r);
#pragma unroll
  for (int i = 0; i < 4; i++) Bf(t, 2 + 4 * i, 3 + 4 * i, 32, 1);
  adst_out_perm<4>(t);
}

// txfm_types::Detail::inverse + INV_TXFM_FNS (inverse.rs:1580-1623), in place
template <int KIND, int N>
RV_DI void inv1d(T *t, int range) {
  if constexpr (KIND == 0) {  // av1_iidentity4/8/16/32 (inverse.rs:111-854)
#pragma unroll
    for (int i = 0; i < N; i++) {
      if constexpr (N == 4) t[i] = round_shift(wmul24(5793, t[i]), 12);
      else if constexpr (N == 8) t[i] = wmul(2, t[i]);
      else if constexpr (N == 16) t[i] = round_shift(wmul24(5793 * 2, t[i]), 12);
      else t[i] = wmul(4, t[i]);
    }
  } else if constexpr (KIND == 1) {
    idct<lg2<N>()>(t, range);
  } else {
    if constexpr (N == 4) iadst4(t);
    else if constexpr (N == 8) iadst8(t, range);
    else iadst16(t, range);
  }
}

}  // namespace tx

// TxSize geometry (src/transform/mod.rs:256-290) and TxType -> 1-D kinds
// (src/transform/mod.rs:158-219), kinds in TBL_IDX order.
__host__ __device__ constexpr int tx_w_log2(int s) {
  constexpr int v[19] = {2, 3, 4, 5, 6, 2, 3, 3, 4, 4, 5, 5, 6, 2, 4, 3, 5, 4, 6};
  return v[s];
}
__host__ __device__ constexpr int tx_h_log2(int s) {
  constexpr int v[19] = {2, 3, 4, 5, 6, 3, 2, 4, 3, 5, 4, 6, 5, 4, 2, 5, 3, 6, 4};
  return v[s];
}
__host__ __device__ constexpr int tx_col_kind(int t) {
  constexpr int v[16] = {1, 2, 1, 2, 3, 1, 3, 2, 3, 0, 1, 0, 2, 0, 3, 0};
  return v[t];
}
__host__ __device__ constexpr int tx_row_kind(int t) {
  constexpr int v[16] = {1, 1, 2, 2, 1, 3, 3, 3, 2, 0, 0, 1, 0, 2, 0, 3};
  return v[t];
}

}  // namespace rv
