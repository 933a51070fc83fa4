// rv_device.h -- device-side primitives shared by the gfx950 kernels.
//
// Integer semantics follow the reference's Rust release build: i32
// arithmetic wraps (done through u32 here to stay clear of C++ UB), `>>` on
// signed values is arithmetic.  Citations: geobacter-rs/rav1e.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/rav1e_hip.h"

#define RV_WAVE 64

namespace rv {

// The work-item id, opaque to loop-invariant code motion: a workgroup that
// loops over work items (rdo_quad_list_kernel) would otherwise compute every
// lane-dependent LDS / pixel offset of the inlined bodies once before the
// loop and keep them all live -- spilled to scratch (~0.5 KB per lane).
__device__ __forceinline__ unsigned rv_tid() {
  unsigned t = threadIdx.x;
  asm volatile("" : "+v"(t));
  return t;
}

__device__ __forceinline__ int32_t wadd(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a + (uint32_t)b);
}
__device__ __forceinline__ int32_t wsub(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a - (uint32_t)b);
}
__device__ __forceinline__ int32_t wmul(int32_t a, int32_t b) {
  return (int32_t)((uint32_t)a * (uint32_t)b);
}
// Wrapping i32 product of operands that fit signed 24 bits: v_mul_i32_i24
// returns the low 32 bits of the exact product, i.e. wmul, at full VALU rate
// (v_mul_lo_u32 is a multi-pass op).  The transforms' data operands stay
// below 2^21 for every i16 residual / clamped coefficient input at 8-12 bits
// (tools/txbounds.c measures them over the oracle), the constants below 2^16.
__device__ __forceinline__ int32_t wmul24(int32_t a, int32_t b) {
  return __mul24(a, b);
}
// Signed integer dot products (v_dot4_i32_i8 / v_dot2_i32_i16).  These stay
// compiler builtins: gfx950 requires wait states between a dot that writes a
// VGPR and another VALU reading it, which the compiler inserts for the
// builtins but cannot see inside inline asm (measured: wrong sub-pel SADs).
__device__ __forceinline__ int32_t dot4_i8(uint32_t a, uint32_t b, int32_t c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}
__device__ __forceinline__ int32_t dot2_i16(uint32_t a, uint32_t b, int32_t c) {
  typedef short s2 __attribute__((ext_vector_type(2)));
  return __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, a), __builtin_bit_cast(s2, b), c, false);
}
// clamp of a signed value into [lo, hi], lo <= hi: one v_med3_i32 (the
// compiler only forms it when both bounds are constants)
__device__ __forceinline__ int32_t clamp_med3(int32_t v, int32_t lo, int32_t hi) {
  int32_t d;
  asm("v_med3_i32 %0, %1, %2, %3" : "=v"(d) : "v"(v), "v"(lo), "v"(hi));
  return d;
}
// round_shift (src/util/mod.rs:241-243); ISimd::round_shift is identical
// (src/util/simd.rs:98-100).  Wrapping add, arithmetic shift.
__device__ __forceinline__ int32_t round_shift(int32_t v, int bit) {
  return wadd(v, (1 << bit) >> 1) >> bit;
}
__host__ __device__ __forceinline__ int32_t clampi(int32_t v, int32_t lo, int32_t hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}
// msb (src/util/mod.rs:235-238)
__device__ __forceinline__ int msb(int32_t x) {
  return 31 - __builtin_clz((uint32_t)x);
}

// Plane addressing (PlaneConfig, src/frame/plane.rs:22-47).
struct PlaneView {
  uint8_t *data;
  int32_t stride;
  int32_t hbd;
  __device__ __forceinline__ int64_t idx(int32_t x, int32_t y) const {
    return (int64_t)y * stride + x;
  }
};

__host__ __device__ __forceinline__ int64_t plane_origin_index(
    const rv_plane &p) {
  return (int64_t)p.yorigin * p.stride + p.xorigin;
}

template <typename Px>
__device__ __forceinline__ const Px *plane_ptr(const rv_plane &p, int32_t x,
                                               int32_t y) {
  return reinterpret_cast<const Px *>(p.data) + plane_origin_index(p) +
         (int64_t)y * p.stride + x;
}
template <typename Px>
__device__ __forceinline__ Px *plane_ptr_mut(const rv_plane &p, int32_t x,
                                             int32_t y) {
  return reinterpret_cast<Px *>(p.data) + plane_origin_index(p) +
         (int64_t)y * p.stride + x;
}

// Wave-level reductions over aligned sub-groups of G lanes (G power of 2,
// <= 64): every lane of the group ends up with the group's total.
template <int G, typename T>
__device__ __forceinline__ T group_sum(T v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, RV_WAVE);
  return v;
}

// Unaligned 4-byte load of u8 pixels (the compiler picks byte loads if the
// target cannot do it in one access).
__device__ __forceinline__ uint32_t load_u32_unaligned(const uint8_t *p) {
  uint32_t v;
  __builtin_memcpy(&v, p, 4);
  return v;
}

// |a - b| summed over the 4 bytes of a and b, plus acc (v_sad_u8).
__device__ __forceinline__ uint32_t sad_u8x4(uint32_t a, uint32_t b,
                                             uint32_t acc) {
  return __builtin_amdgcn_sad_u8(a, b, acc);
}

// ---- SATD chunk: get_satd_ref (src/dist.rs:197-328) ------------------------
// The butterfly network is exact integer arithmetic whose outputs are a
// signed permutation of the Walsh-Hadamard transform, so sum |.| does not
// depend on butterfly order; the network below is the reference's
// (hadamard4_1d / hadamard8_1d, src/dist.rs:208-256).
template <int N>
__device__ __forceinline__ void had1d(int32_t *v, int s) {
#pragma unroll
  for (int k = 0; k < N; k += 2) {
    int32_t a = v[k * s], b = v[(k + 1) * s];
    v[k * s] = a + b;
    v[(k + 1) * s] = a - b;
  }
#pragma unroll
  for (int g = 0; g < N; g += 4)
#pragma unroll
    for (int k = 0; k < 2; k++) {
      int32_t a = v[(g + k) * s], b = v[(g + k + 2) * s];
      v[(g + k) * s] = a + b;
      v[(g + k + 2) * s] = a - b;
    }
  if constexpr (N == 8) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      int32_t a = v[k * s], b = v[(k + 4) * s];
      v[k * s] = a + b;
      v[(k + 4) * s] = a - b;
    }
  }
}

// Order the LDS accesses of one wavefront's lanes (no workgroup barrier).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int N>
__device__ __forceinline__ uint64_t satd_chunk(int32_t *d) {
#pragma unroll
  for (int c = 0; c < N; c++) had1d<N>(d + c, N);  // vertical
#pragma unroll
  for (int r = 0; r < N; r++) had1d<N>(d + r * N, 1);  // horizontal
  uint32_t s = 0;  // <= 64 * 64 * 4095 per 8x8 chunk: fits u32
#pragma unroll
  for (int i = 0; i < N * N; i++) s += (uint32_t)(d[i] < 0 ? -d[i] : d[i]);
  return s;
}

}  // namespace rv

#define RV_HIP_CHECK_LAUNCH()                                   \
  do {                                                          \
    hipError_t e_ = hipGetLastError();                          \
    if (e_ != hipSuccess) return rv_set_hip_error(e_, __func__); \
  } while (0)

// Host-side helpers implemented in rv_runtime.cpp.
extern "C++" int rv_set_hip_error(hipError_t e, const char *where);
extern "C++" int rv_set_error(int code, const char *msg);
extern "C++" hipStream_t rv_resolve_stream(void *stream);
