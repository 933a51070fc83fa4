// rv_shims.hip -- layer 1 of include/rav1e_hip.h: per-call entry points
// with the reference's asm FFI signatures (src/asm/x86/dist.rs:16-98,
// src/asm/x86/mc.rs:17-78) and the [cpu][index] dispatch tables.
//
// Each call stages its block(s) (host memory, byte strides) through pinned
// memory into one device scratch buffer, runs the batched kernel with n = 1
// on the calling thread's own stream and copies the result back.  Thread
// local state keeps the calls reentrant across rayon-style worker threads.
// There is no error channel in these signatures (there is none in NASM
// either): a HIP failure prints and aborts, it never returns a wrong value.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "rv_device.h"

namespace {

// Per-thread staging context.  It has no destructor on purpose: a
// thread_local destructor runs at thread / process exit, possibly after the
// HIP runtime has been torn down (a known crash-at-exit of drop-in asm
// backends).  Contexts are released explicitly by rv_shims_release() (the
// calling thread's) or rv_shims_shutdown() (all of them), and are otherwise
// left to the process teardown.
struct ShimCtx {
  hipStream_t stream = nullptr;
  uint8_t *dev = nullptr;
  uint8_t *host = nullptr;
  size_t cap = 0;
};
thread_local ShimCtx *g_ctx = nullptr;
std::mutex g_all_mu;
std::vector<ShimCtx *> g_all;

void free_ctx(ShimCtx *c) {
  if (c->dev) (void)hipFree(c->dev);
  if (c->host) (void)hipHostFree(c->host);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

[[noreturn]] void die(const char *what, const char *detail) {
  fprintf(stderr, "rav1e_hip: %s failed: %s\n", what, detail);
  abort();
}
void check(hipError_t e, const char *what) {
  if (e != hipSuccess) die(what, hipGetErrorString(e));
}
void check_rv(int rc, const char *what) {
  if (rc != RV_OK) die(what, rv_last_error());
}

ShimCtx &ctx(size_t bytes) {
  if (!g_ctx) {
    g_ctx = new ShimCtx();
    std::lock_guard<std::mutex> lk(g_all_mu);
    g_all.push_back(g_ctx);
  }
  ShimCtx &c = *g_ctx;
  if (!c.stream) check(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking),
                       "hipStreamCreate");
  if (bytes > c.cap) {
    size_t cap = 1 << 16;
    while (cap < bytes) cap <<= 1;
    if (c.dev) check(hipFree(c.dev), "hipFree");
    if (c.host) check(hipHostFree(c.host), "hipHostFree");
    check(hipMalloc(&c.dev, cap), "hipMalloc");
    check(hipHostMalloc(&c.host, cap, hipHostMallocDefault), "hipHostMalloc");
    c.cap = cap;
  }
  return c;
}

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

// Copy a w x h region (element size px, byte stride) into packed rows.
void pack(uint8_t *dst, const void *src, ptrdiff_t stride, int w, int h,
          int px) {
  for (int r = 0; r < h; r++)
    memcpy(dst + (size_t)r * w * px, (const uint8_t *)src + r * stride,
           (size_t)w * px);
}
void unpack(void *dst, ptrdiff_t stride, const uint8_t *src, int w, int h,
            int px) {
  for (int r = 0; r < h; r++)
    memcpy((uint8_t *)dst + r * stride, src + (size_t)r * w * px,
           (size_t)w * px);
}

rv_plane packed_plane(void *data, int w, int h, int margin, int hbd) {
  rv_plane p;
  memset(&p, 0, sizeof(p));
  p.data = data;
  p.stride = w + 2 * margin + (margin ? 1 : 0);
  p.alloc_height = h + 2 * margin + (margin ? 1 : 0);
  p.width = w;
  p.height = h;
  p.xorigin = margin;
  p.yorigin = margin;
  p.hbd = hbd;
  return p;
}

// SAD / SATD of one block: src, dst = the two regions (byte strides).
uint32_t dist_call(int metric, const void *src, ptrdiff_t ss, const void *dst,
                   ptrdiff_t ds, int w, int h, int hbd) {
  const int px = hbd ? 2 : 1;
  const size_t blk = align256((size_t)w * h * px);
  const size_t off_b = blk, off_job = 2 * blk, off_out = off_job + 256;
  ShimCtx &c = ctx(off_out + 256);
  pack(c.host, src, ss, w, h, px);
  pack(c.host + off_b, dst, ds, w, h, px);
  rv_dist_job job{0, 0, 0, 0};
  memcpy(c.host + off_job, &job, sizeof(job));
  check(hipMemcpyAsync(c.dev, c.host, off_out, hipMemcpyHostToDevice, c.stream),
        "hipMemcpyAsync");
  rv_plane a = packed_plane(c.dev, w, h, 0, hbd);
  rv_plane b = packed_plane(c.dev + off_b, w, h, 0, hbd);
  const rv_dist_job *dj = (const rv_dist_job *)(c.dev + off_job);
  uint32_t *dout = (uint32_t *)(c.dev + off_out);
  check_rv(metric ? rv_satd_batch(&a, &b, dj, 1, w, h, dout, c.stream)
                  : rv_sad_batch(&a, &b, dj, 1, w, h, dout, c.stream),
           metric ? "rv_satd_batch" : "rv_sad_batch");
  uint32_t out = 0;
  check(hipMemcpyAsync(&out, dout, 4, hipMemcpyDeviceToHost, c.stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
  return out;
}

// put / prep of one block; src points at the block's integer position.
void mc_call(int prep, void *dst, ptrdiff_t dst_stride, const void *src,
             ptrdiff_t src_stride, int w, int h, int mx, int my, int mode_x,
             int mode_y, int bd, int hbd) {
  const int px = hbd ? 2 : 1;
  rv_plane sp = packed_plane(nullptr, w, h, 3, hbd);  // rows/cols -3..+4
  const size_t sbytes = align256((size_t)sp.stride * sp.alloc_height * px);
  const size_t obytes = align256((size_t)w * h * (prep ? 2 : px));
  const size_t off_out = sbytes, off_job = sbytes + obytes;
  ShimCtx &c = ctx(off_job + 256);
  pack(c.host, (const uint8_t *)src - 3 * src_stride - 3 * px, src_stride,
       sp.stride, sp.alloc_height, px);
  rv_mc_job job{0, 0, 0, 0, mx, my};
  memcpy(c.host + off_job, &job, sizeof(job));
  check(hipMemcpyAsync(c.dev, c.host, off_job + 256, hipMemcpyHostToDevice,
                       c.stream),
        "hipMemcpyAsync");
  sp.data = c.dev;
  const rv_mc_job *dj = (const rv_mc_job *)(c.dev + off_job);
  if (prep) {
    check_rv(rv_prep_8tap_batch((int16_t *)(c.dev + off_out), &sp, dj, 1, w, h,
                                mode_x, mode_y, bd, c.stream),
             "rv_prep_8tap_batch");
  } else {
    rv_plane dp = packed_plane(c.dev + off_out, w, h, 0, hbd);
    check_rv(rv_put_8tap_batch(&dp, &sp, dj, 1, w, h, mode_x, mode_y, bd,
                               c.stream),
             "rv_put_8tap_batch");
  }
  check(hipMemcpyAsync(c.host + off_out, c.dev + off_out, obytes,
                       hipMemcpyDeviceToHost, c.stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
  if (prep)
    memcpy(dst, c.host + off_out, (size_t)w * h * 2);
  else
    unpack(dst, dst_stride, c.host + off_out, w, h, px);
}

void avg_call(void *dst, ptrdiff_t dst_stride, const int16_t *t1,
              const int16_t *t2, int w, int h, int bd, int hbd) {
  const int px = hbd ? 2 : 1;
  const size_t tb = align256((size_t)w * h * 2);
  const size_t off_job = 2 * tb, off_out = off_job + 256;
  const size_t obytes = align256((size_t)w * h * px);
  ShimCtx &c = ctx(off_out + obytes);
  memcpy(c.host, t1, (size_t)w * h * 2);
  memcpy(c.host + tb, t2, (size_t)w * h * 2);
  rv_mc_job job{0, 0, 0, 0, 0, 0};
  memcpy(c.host + off_job, &job, sizeof(job));
  check(hipMemcpyAsync(c.dev, c.host, off_out, hipMemcpyHostToDevice, c.stream),
        "hipMemcpyAsync");
  rv_plane dp = packed_plane(c.dev + off_out, w, h, 0, hbd);
  check_rv(rv_mc_avg_batch(&dp, (const int16_t *)c.dev,
                           (const int16_t *)(c.dev + tb),
                           (const rv_mc_job *)(c.dev + off_job), 1, w, h, bd,
                           c.stream),
           "rv_mc_avg_batch");
  check(hipMemcpyAsync(c.host + off_out, c.dev + off_out, obytes,
                       hipMemcpyDeviceToHost, c.stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
  unpack(dst, dst_stride, c.host + off_out, w, h, px);
}

constexpr int kTxW[19] = {4, 8, 16, 32, 64, 4, 8, 8, 16, 16, 32, 32, 64, 4, 16, 8, 32, 16, 64};
constexpr int kTxH[19] = {4, 8, 16, 32, 64, 8, 4, 16, 8, 32, 16, 64, 32, 16, 4, 32, 8, 64, 16};

}  // namespace

extern "C" {

#define RV_DEF_DIST(W, H)                                                     \
  uint32_t rav1e_sad##W##x##H##_hip(const uint8_t *src, ptrdiff_t ss,          \
                                    const uint8_t *dst, ptrdiff_t ds) {       \
    return dist_call(0, src, ss, dst, ds, W, H, 0);                           \
  }                                                                           \
  uint32_t rav1e_sad##W##x##H##_hbd_hip(const uint16_t *src, ptrdiff_t ss,     \
                                        const uint16_t *dst, ptrdiff_t ds) {  \
    return dist_call(0, src, ss, dst, ds, W, H, 1);                           \
  }                                                                           \
  uint32_t rav1e_satd_##W##x##H##_hip(const uint8_t *src, ptrdiff_t ss,        \
                                      const uint8_t *dst, ptrdiff_t ds) {     \
    return dist_call(1, src, ss, dst, ds, W, H, 0);                           \
  }                                                                           \
  uint32_t rav1e_satd_##W##x##H##_hbd_hip(const uint16_t *src, ptrdiff_t ss,   \
                                          const uint16_t *dst, ptrdiff_t ds) { \
    return dist_call(1, src, ss, dst, ds, W, H, 1);                           \
  }
RV_DIST_SIZES(RV_DEF_DIST)
#undef RV_DEF_DIST

#define RV_DEF_MC(NX, NY, MX, MY)                                              \
  void rav1e_put_8tap_##NX##_##NY##_hip(uint8_t *dst, ptrdiff_t ds,            \
                                        const uint8_t *src, ptrdiff_t ss,      \
                                        int32_t w, int32_t h, int32_t mx,      \
                                        int32_t my) {                          \
    mc_call(0, dst, ds, src, ss, w, h, mx, my, MX, MY, 8, 0);                  \
  }                                                                            \
  void rav1e_put_8tap_##NX##_##NY##_16bpc_hip(                                 \
      uint16_t *dst, ptrdiff_t ds, const uint16_t *src, ptrdiff_t ss,          \
      int32_t w, int32_t h, int32_t mx, int32_t my, int32_t bd) {              \
    mc_call(0, dst, ds, src, ss, w, h, mx, my, MX, MY, bd, 1);                 \
  }                                                                            \
  void rav1e_prep_8tap_##NX##_##NY##_hip(int16_t *tmp, const uint8_t *src,     \
                                         ptrdiff_t ss, int32_t w, int32_t h,   \
                                         int32_t mx, int32_t my) {             \
    mc_call(1, tmp, 0, src, ss, w, h, mx, my, MX, MY, 8, 0);                   \
  }                                                                            \
  void rav1e_prep_8tap_##NX##_##NY##_16bpc_hip(                                \
      int16_t *tmp, const uint16_t *src, ptrdiff_t ss, int32_t w, int32_t h,   \
      int32_t mx, int32_t my, int32_t bd) {                                    \
    mc_call(1, tmp, 0, src, ss, w, h, mx, my, MX, MY, bd, 1);                  \
  }
RV_FILTER_PAIRS(RV_DEF_MC)
#undef RV_DEF_MC

void rav1e_avg_hip(uint8_t *dst, ptrdiff_t ds, const int16_t *t1,
                   const int16_t *t2, int32_t w, int32_t h) {
  avg_call(dst, ds, t1, t2, w, h, 8, 0);
}
void rav1e_avg_16bpc_hip(uint16_t *dst, ptrdiff_t ds, const int16_t *t1,
                         const int16_t *t2, int32_t w, int32_t h, int32_t bd) {
  avg_call(dst, ds, t1, t2, w, h, bd, 1);
}

int rav1e_fwd_txfm_hip(const int16_t *residual, int32_t *coeffs,
                       int32_t tx_size, int32_t tx_type, int32_t bd) {
  if (tx_size < 0 || tx_size > 18) return RV_EINVAL;
  const int w = kTxW[tx_size], h = kTxH[tx_size];
  const size_t rb = align256((size_t)w * h * 2), cb = (size_t)w * h * 4;
  ShimCtx &c = ctx(rb + cb);
  memcpy(c.host, residual, (size_t)w * h * 2);
  check(hipMemcpyAsync(c.dev, c.host, rb, hipMemcpyHostToDevice, c.stream),
        "hipMemcpyAsync");
  int rc = rv_fwd_txfm_batch((const int16_t *)c.dev, (int32_t *)(c.dev + rb), 1,
                             tx_size, tx_type, bd, c.stream);
  if (rc != RV_OK) return rc;  // unsupported (size, type) pair
  check(hipMemcpyAsync(c.host + rb, c.dev + rb, cb, hipMemcpyDeviceToHost,
                       c.stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
  memcpy(coeffs, c.host + rb, cb);
  return RV_OK;
}

int rav1e_inv_txfm_add_hip(const int32_t *coeffs, void *dst,
                           ptrdiff_t dst_stride, int32_t tx_size,
                           int32_t tx_type, int32_t bd) {
  if (tx_size < 0 || tx_size > 18) return RV_EINVAL;
  const int w = kTxW[tx_size], h = kTxH[tx_size];
  const int cw = w < 32 ? w : 32, ch = h < 32 ? h : 32;
  const int hbd = bd > 8, px = hbd ? 2 : 1;
  const size_t cb = align256((size_t)cw * ch * 4);
  const size_t db = align256((size_t)w * h * px);
  const size_t off_d = cb, off_job = cb + db;
  ShimCtx &c = ctx(off_job + 256);
  memcpy(c.host, coeffs, (size_t)cw * ch * 4);
  pack(c.host + off_d, dst, dst_stride, w, h, px);
  rv_tx_job job{0, 0, 0, 0};
  memcpy(c.host + off_job, &job, sizeof(job));
  check(hipMemcpyAsync(c.dev, c.host, off_job + 256, hipMemcpyHostToDevice,
                       c.stream),
        "hipMemcpyAsync");
  rv_plane dp = packed_plane(c.dev + off_d, w, h, 0, hbd);
  int rc = rv_inv_txfm_add_batch((const int32_t *)c.dev, &dp,
                                 (const rv_tx_job *)(c.dev + off_job), 1,
                                 tx_size, tx_type, bd, c.stream);
  if (rc != RV_OK) return rc;
  check(hipMemcpyAsync(c.host + off_d, c.dev + off_d, db, hipMemcpyDeviceToHost,
                       c.stream),
        "hipMemcpyAsync");
  check(hipStreamSynchronize(c.stream), "hipStreamSynchronize");
  unpack(dst, dst_stride, c.host + off_d, w, h, px);
  return RV_OK;
}

// ---- dispatch tables (shape of SAD_FNS / SATD_FNS / PUT_FNS) ------------
#define RV_PTR_SAD(W, H) (rv_dist_fn)rav1e_sad##W##x##H##_hip,
#define RV_PTR_SAD_HBD(W, H) (rv_dist_fn)rav1e_sad##W##x##H##_hbd_hip,
#define RV_PTR_SATD(W, H) (rv_dist_fn)rav1e_satd_##W##x##H##_hip,
#define RV_PTR_SATD_HBD(W, H) (rv_dist_fn)rav1e_satd_##W##x##H##_hbd_hip,
static const rv_dist_fn kSad[2][22] = {{RV_DIST_SIZES(RV_PTR_SAD)},
                                       {RV_DIST_SIZES(RV_PTR_SAD_HBD)}};
static const rv_dist_fn kSatd[2][22] = {{RV_DIST_SIZES(RV_PTR_SATD)},
                                        {RV_DIST_SIZES(RV_PTR_SATD_HBD)}};
#define RV_PTR_PUT(NX, NY, MX, MY) (rv_put_fn)rav1e_put_8tap_##NX##_##NY##_hip,
static const rv_put_fn kPut[16] = {RV_FILTER_PAIRS(RV_PTR_PUT)};

rv_dist_fn rv_sad_fn(int cpu_level, int bsize, int hbd) {
  if (cpu_level != RV_CPU_HIP) return nullptr;
  bsize &= 31;  // to_index (src/asm/x86/dist.rs:104-106)
  return bsize < 22 ? kSad[hbd ? 1 : 0][bsize] : nullptr;
}
rv_dist_fn rv_satd_fn(int cpu_level, int bsize, int hbd) {
  if (cpu_level != RV_CPU_HIP) return nullptr;
  bsize &= 31;
  return bsize < 22 ? kSatd[hbd ? 1 : 0][bsize] : nullptr;
}
rv_put_fn rv_put_fn_get(int cpu_level, int mode_x, int mode_y) {
  if (cpu_level != RV_CPU_HIP) return nullptr;
  return kPut[(mode_x + 4 * mode_y) & 15];  // get_2d_mode_idx
}

}  // extern "C"

extern "C" void rv_shims_release(void) {
  if (!g_ctx) return;
  {
    std::lock_guard<std::mutex> lk(g_all_mu);
    for (size_t i = 0; i < g_all.size(); i++)
      if (g_all[i] == g_ctx) {
        g_all.erase(g_all.begin() + (long)i);
        break;
      }
  }
  free_ctx(g_ctx);
  g_ctx = nullptr;
}

extern "C" void rv_shims_shutdown(void) {
  std::lock_guard<std::mutex> lk(g_all_mu);
  for (ShimCtx *c : g_all) free_ctx(c);
  g_all.clear();
  g_ctx = nullptr;  // other threads' pointers are stale: they must not call again
}
