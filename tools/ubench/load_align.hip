// Micro-benchmark: cost of global loads whose lane addresses are not
// naturally aligned (the motion searches read u8 / u16 windows at arbitrary
// offsets).  Each lane reads ITERS rows of W bytes at byte offset OFF from
// a contiguous, L2-resident 4 MiB window (lane i at i * W); reports time per
// wave-load and effective bytes/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define ITERS 256
#define PITCH 4096

template <int W>
__global__ __launch_bounds__(256) void k(const uint8_t *buf, int off, uint32_t *out) {
  const int lane = threadIdx.x & 63, wave = (blockIdx.x * 4 + (threadIdx.x >> 6)) & 1023;
  const uint8_t *p = buf + off + lane * W + (size_t)(wave & 63) * 64 * W;
  uint32_t acc = 0;
#pragma unroll 8
  for (int it = 0; it < ITERS; it++) {
    const uint8_t *q = p + (size_t)((it + wave) & 1023) * PITCH;
    if constexpr (W == 4) {
      uint32_t v;
      __builtin_memcpy(&v, q, 4);
      acc += v;
    } else if constexpr (W == 8) {
      uint2 v;
      __builtin_memcpy(&v, q, 8);
      acc += v.x ^ v.y;
    } else {
      uint4 v;
      __builtin_memcpy(&v, q, 16);
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <int W>
static void run(const uint8_t *buf, uint32_t *out, int off) {
  const int blocks = 256 * 8;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  k<W><<<blocks, 256>>>(buf, off, out);
  hipEventRecord(a);
  for (int r = 0; r < 5; r++) k<W><<<blocks, 256>>>(buf, off, out);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  const double waveloads = 5.0 * blocks * 4 * ITERS;
  const double t = ms / 1e3;
  printf("W=%2d off=%d: %.3f ms  %.2f ns/wave-load/CU  %.1f GB/s\n", W, off, ms / 5,
         t / waveloads * 256 * 1e9, waveloads * 64 * W / t / 1e9);
}

int main() {
  uint8_t *buf;
  uint32_t *out;
  hipMalloc(&buf, (size_t)1024 * PITCH + 4096 * 64);
  hipMemset(buf, 1, (size_t)1024 * PITCH + 4096 * 64);
  hipMalloc(&out, 64);
  for (int off : {0, 1, 2, 4, 8}) {
    run<4>(buf, out, off);
    run<8>(buf, out, off);
    run<16>(buf, out, off);
  }
  return 0;
}
