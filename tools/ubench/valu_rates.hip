// Micro-benchmark: issue rate of the integer VALU instructions the SAD /
// filter kernels are built from (v_sad_u8, v_msad_u8, v_qsad_pk_u16_u8,
// v_mqsad_u32_u8, v_dot4_i32_i8, v_dot2_i32_i16, v_mad_i32_i24, v_add_u32)
// on gfx950: many independent accumulator chains per lane, wave64, full
// occupancy; reports wave-instructions per cycle per CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define ITERS 4096
#define CHAINS 8

template <int OP>
__global__ __launch_bounds__(256) void k(uint32_t *out, uint32_t seed) {
  uint32_t a[CHAINS];
  uint64_t q[CHAINS / 4];
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  u4 qa[CHAINS / 4];
  for (int i = 0; i < CHAINS; i++) a[i] = seed * (threadIdx.x + i);
  for (int i = 0; i < CHAINS / 4; i++) { q[i] = ((uint64_t)seed << 32) | (threadIdx.x * 77 + i); qa[i] = (u4){a[i], a[i+1], 3, 4}; }
  uint32_t b = seed ^ threadIdx.x, c = seed + 17 * threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < CHAINS; i++) {
      if constexpr (OP == 0) a[i] = __builtin_amdgcn_sad_u8(b, c + i, a[i]);
      if constexpr (OP == 1) a[i] = __builtin_amdgcn_msad_u8(b, c + i, a[i]);
      if constexpr (OP == 2) a[i] = __builtin_amdgcn_sdot4((int)b, (int)(c + i), (int)a[i], false);
      if constexpr (OP == 3) {
        typedef short s2 __attribute__((ext_vector_type(2)));
        a[i] = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2, b), __builtin_bit_cast(s2, c + i), (int)a[i], false);
      }
      // dependent on the accumulator, so the compiler cannot hoist or fold
      // the loop (8 independent chains per lane, 8 waves per SIMD)
      if constexpr (OP == 4) a[i] = __mul24((int)a[i], (int)(c + i)) + b;
      if constexpr (OP == 5) a[i] = (a[i] ^ b) + c;
      if constexpr (OP == 6) a[i] = __builtin_amdgcn_alignbyte(b, a[i], c);
    }
    if constexpr (OP == 7) {
#pragma unroll
      for (int i = 0; i < CHAINS / 4; i++) q[i] = __builtin_amdgcn_qsad_pk_u16_u8(q[i] ^ b, c + i, q[i]);
    }
    if constexpr (OP == 8) {
#pragma unroll
      for (int i = 0; i < CHAINS / 4; i++) qa[i] = __builtin_amdgcn_mqsad_u32_u8(((uint64_t)b << 32) | c, c + i, qa[i]);
    }
  }
  uint32_t s = 0;
  for (int i = 0; i < CHAINS; i++) s += a[i];
  for (int i = 0; i < CHAINS / 4; i++) s += (uint32_t)q[i] + qa[i].x + qa[i].w;
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int OP>
void run(const char *name, int per_iter, uint32_t *d, int ncu) {
  const int blocks = ncu * 8;  // 32 waves per CU
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  k<OP><<<blocks, 256>>>(d, 1);
  hipEventRecord(e0);
  k<OP><<<blocks, 256>>>(d, 3);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double winstr = (double)blocks * 4 * ITERS * per_iter;
  const double clk = 2.4e9;
  printf("%-18s %8.3f ms  %6.3f wave-instr/cycle/CU  (%.1f lane-ops/clk/CU at 2.4 GHz)\n", name, ms,
         winstr / (ms * 1e-3 * clk) / ncu, winstr * 64 / (ms * 1e-3 * clk) / ncu);
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  printf("%s, %d CUs, clock %d kHz\n", p.gcnArchName, ncu, p.clockRate);
  uint32_t *d;
  hipMalloc(&d, (size_t)ncu * 8 * 256 * 4);
  run<0>("v_sad_u8", CHAINS, d, ncu);
  run<1>("v_msad_u8", CHAINS, d, ncu);
  run<2>("v_dot4_i32_i8", CHAINS, d, ncu);
  run<3>("v_dot2_i32_i16", CHAINS, d, ncu);
  run<4>("v_mad_i32_i24", CHAINS, d, ncu);
  run<5>("v_add+xor", 2 * CHAINS, d, ncu);
  run<6>("v_alignbyte", CHAINS, d, ncu);
  run<7>("v_qsad_pk_u16_u8", CHAINS / 4, d, ncu);
  run<8>("v_mqsad_u32_u8", CHAINS / 4, d, ncu);
  return 0;
}
