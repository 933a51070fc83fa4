// PMC calibration: kernels with known byte counts, run under
//   rocprofv3 --pmc FETCH_SIZE   and   rocprofv3 --pmc WRITE_SIZE
// to derive the per-access-width factors of gfx950's FETCH_SIZE /
// WRITE_SIZE (MI355X_MICROARCH.md: only 16-B streaming reads are
// calibrated there).  Buffers are 1 GiB, past the 256 MiB Infinity Cache.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr size_t kBytes = 1ull << 30;

__global__ void rd_dword(const uint32_t *__restrict__ a, uint32_t *__restrict__ o, size_t n) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 0x12345678) o[0] = s;
}
__global__ void rd_x4(const uint4 *__restrict__ a, uint32_t *__restrict__ o, size_t n) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    uint4 v = a[i];
    s += v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678) o[0] = s;
}
__global__ void rd_byte(const uint8_t *__restrict__ a, uint32_t *__restrict__ o, size_t n) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += a[i];
  if (s == 0x12345678) o[0] = s;
}
__global__ void wr_dword(uint32_t *__restrict__ o, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) o[i] = (uint32_t)i;
}
__global__ void wr_x4(uint4 *__restrict__ o, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    o[i] = make_uint4((uint32_t)i, 1, 2, 3);
}
__global__ void wr_byte(uint8_t *__restrict__ o, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) o[i] = (uint8_t)i;
}

int main() {
  void *a, *o;
  hipMalloc(&a, kBytes);
  hipMalloc(&o, kBytes);
  hipMemset(a, 1, kBytes);
  const int grid = 256 * 16;
  for (int rep = 0; rep < 2; rep++) {
    rd_dword<<<grid, 256>>>((const uint32_t *)a, (uint32_t *)o, kBytes / 4);
    rd_x4<<<grid, 256>>>((const uint4 *)a, (uint32_t *)o, kBytes / 16);
    rd_byte<<<grid, 256>>>((const uint8_t *)a, (uint32_t *)o, kBytes);
    wr_dword<<<grid, 256>>>((uint32_t *)o, kBytes / 4);
    wr_x4<<<grid, 256>>>((uint4 *)o, kBytes / 16);
    wr_byte<<<grid, 256>>>((uint8_t *)o, kBytes);
  }
  hipDeviceSynchronize();
  printf("each kernel moves %zu bytes (1 GiB)\n", kBytes);
  return 0;
}
