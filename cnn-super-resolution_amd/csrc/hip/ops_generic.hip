// ops_generic.hip -- runtime-shape HIP kernels for every reference operator.
//
// These are the shape-generic implementations behind srcnn.h: they accept any
// (n_prev, n_cur, f, w, h, batch) the reference accepts, keep the reference's
// per-output accumulation order, and are the fallback whenever no gfx950
// specialisation (ops_fast.hip) matches the shape.  One thread computes one
// output element; consecutive lanes take consecutive channels, so loads and
// stores of the HWC activations coalesce.
#include "common.hpp"
#include "ops.hpp"

namespace srcnn {
namespace generic {

// ---------------------------------------------------------------------------
// forward: src/kernel/layer_uber_kernel.cl:36-96
// ---------------------------------------------------------------------------
__global__ void conv_fwd_kernel(const float* __restrict__ in, float* __restrict__ out,
                                const float* __restrict__ W, const float* __restrict__ B,
                                uint32_t in_w, uint32_t in_h, uint32_t n_prev,
                                uint32_t n_cur, uint32_t f, int relu, size_t total) {
  const uint32_t out_w = in_w - f + 1, out_h = in_h - f + 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t n = i % n_cur;
    size_t t = i / n_cur;
    const uint32_t x = t % out_w;
    t /= out_w;
    const uint32_t y = t % out_h;
    const size_t s = t / out_h;
    const float* img = in + s * n_prev * in_w * in_h;
    float acc = 0.0f;
    for (uint32_t dy = 0; dy < f; dy++)
      for (uint32_t dx = 0; dx < f; dx++) {
        const float* px = img + ((size_t)(y + dy) * in_w + (x + dx)) * n_prev;
        const float* w = W + (size_t)(dy * f + dx) * n_cur * n_prev + n;
        for (uint32_t k = 0; k < n_prev; k++) acc += w[(size_t)k * n_cur] * px[k];
      }
    const float r = acc + B[n];
    out[i] = relu ? fmaxf(r, 0.0f) : r;
  }
}

int conv_fwd(const float* in, float* out, const float* W, const float* B, uint32_t in_w,
             uint32_t in_h, uint32_t n_prev, uint32_t n_cur, uint32_t f, int relu,
             uint32_t batch, hipStream_t s) {
  const size_t total = (size_t)batch * (in_w - f + 1) * (in_h - f + 1) * n_cur;
  SRCNN_PROFILE("conv_fwd_generic", s);
  hipLaunchKernelGGL(conv_fwd_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, in, out, W,
                     B, in_w, in_h, n_prev, n_cur, f, relu, total);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// ---------------------------------------------------------------------------
// last layer delta: src/kernel/last_layer_delta.cl:14-50
// ---------------------------------------------------------------------------
__global__ void last_delta_kernel(const float* __restrict__ gt, const float* __restrict__ y,
                                  float* __restrict__ d, uint32_t gt_w, uint32_t gt_h,
                                  uint32_t out_w, uint32_t out_h, size_t total) {
  const uint32_t pad = (gt_w - out_w) / 2;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t c = i % out_w;
    size_t t = i / out_w;
    const uint32_t r = t % out_h;
    const size_t s = t / out_h;
    const float tv = gt[s * gt_w * gt_h + (size_t)(r + pad) * gt_w + pad + c];
    const float v = y[i];
    d[i] = (v - tv) * (v > 0.0f ? 1.0f : 0.0f);
  }
}

int last_delta(const float* gt, const float* y, float* d, uint32_t gt_w, uint32_t gt_h,
               uint32_t out_w, uint32_t out_h, uint32_t batch, hipStream_t s) {
  const size_t total = (size_t)batch * out_w * out_h;
  SRCNN_PROFILE("last_delta", s);
  hipLaunchKernelGGL(last_delta_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, gt, y, d,
                     gt_w, gt_h, out_w, out_h, total);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// ---------------------------------------------------------------------------
// deltas: src/kernel/layer_deltas.cl:42-127
// ---------------------------------------------------------------------------
__global__ void conv_delta_kernel(const float* __restrict__ d_next,
                                  const float* __restrict__ y_curr, float* __restrict__ d_curr,
                                  const float* __restrict__ W, uint32_t f_next,
                                  uint32_t n_curr, uint32_t n_next, uint32_t curr_w,
                                  uint32_t curr_h, size_t total) {
  const int next_w = (int)curr_w - (int)f_next + 1, next_h = (int)curr_h - (int)f_next + 1;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t n = i % n_curr;
    size_t t = i / n_curr;
    const int x = t % curr_w;
    t /= curr_w;
    const int y = t % curr_h;
    const size_t s = t / curr_h;
    const float deriv = y_curr[i] > 0.0f ? 1.0f : 0.0f;
    const float* dn = d_next + s * n_next * (size_t)next_w * next_h;
    float acc = 0.0f;
    for (int dy = 0; dy < (int)f_next; dy++)
      for (int dx = 0; dx < (int)f_next; dx++) {
        const int nx = x - dx, ny = y - dy;
        if (nx < 0 || nx >= next_w || ny < 0 || ny >= next_h) continue;  // adds 0
        const float* dp = dn + ((size_t)ny * next_w + nx) * n_next;
        const float* w = W + ((size_t)(dy * f_next + dx) * n_curr + n) * n_next;
        for (uint32_t k = 0; k < n_next; k++) acc += dp[k] * w[k] * deriv;
      }
    d_curr[i] = acc;
  }
}

int conv_delta(const float* d_next, const float* y_curr, float* d_curr, const float* W_next,
               uint32_t f_next, uint32_t n_curr, uint32_t n_next, uint32_t curr_w,
               uint32_t curr_h, uint32_t batch, hipStream_t s) {
  const size_t total = (size_t)batch * curr_w * curr_h * n_curr;
  SRCNN_PROFILE("conv_delta_generic", s);
  hipLaunchKernelGGL(conv_delta_kernel, dim3(grid_for(total, 256)), dim3(256), 0, s, d_next,
                     y_curr, d_curr, W_next, f_next, n_curr, n_next, curr_w, curr_h, total);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// ---------------------------------------------------------------------------
// gradients: src/kernel/backpropagate.cl:56-114, race-free.
// Pass 1: one thread per (weight-or-bias item, sample) writes that sample's
//         sum over output pixels (the reference work-item, :89-106).
// Pass 2: one thread per item adds the per-sample sums in sample order.
// ---------------------------------------------------------------------------
__global__ void grad_partial_kernel(const float* __restrict__ in, const float* __restrict__ d,
                                    float* __restrict__ part, uint32_t n_prev, uint32_t n_cur,
                                    uint32_t f, uint32_t out_w, uint32_t out_h,
                                    uint32_t s0, uint32_t chunk) {
  const uint32_t nW = f * f * n_prev * n_cur;
  const uint32_t per = nW + n_cur;
  const uint32_t in_w = out_w + f - 1, in_h = out_h + f - 1;
  const size_t total = (size_t)per * chunk;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const uint32_t item = i % per;
    const uint32_t sl = i / per;
    const size_t s = (size_t)s0 + sl;
    const float* dl = d + s * n_cur * out_w * out_h;
    float acc = 0.0f;
    if (item < nW) {
      uint32_t t = item;
      const uint32_t n = t % n_cur;  // id decode, backpropagate.cl:78-85
      t /= n_cur;
      const uint32_t k = t % n_prev;
      t /= n_prev;
      const uint32_t dx = t % f;
      const uint32_t dy = t / f;
      const float* img = in + s * n_prev * in_w * in_h;
      for (uint32_t row = 0; row < out_h; row++)
        for (uint32_t col = 0; col < out_w; col++) {
          const float delta = dl[((size_t)row * out_w + col) * n_cur + n];
          const float v = img[((size_t)(row + dy) * in_w + (col + dx)) * n_prev + k];
          acc += v * delta;
        }
    } else {
      const uint32_t n = item - nW;
      for (uint32_t p = 0; p < out_w * out_h; p++) acc += dl[(size_t)p * n_cur + n];
    }
    part[(size_t)sl * per + item] = acc;
  }
}

__global__ void grad_reduce_kernel(const float* __restrict__ part, float* __restrict__ gW,
                                   float* __restrict__ gB, uint32_t nW, uint32_t n_cur,
                                   uint32_t chunk) {
  const uint32_t per = nW + n_cur;
  for (uint32_t item = blockIdx.x * blockDim.x + threadIdx.x; item < per;
       item += gridDim.x * blockDim.x) {
    float* dst = item < nW ? gW + item : gB + (item - nW);
    float acc = *dst;
    for (uint32_t s = 0; s < chunk; s++) acc += part[(size_t)s * per + item];
    *dst = acc;
  }
}

size_t grad_workspace_bytes(uint32_t n_prev, uint32_t n_cur, uint32_t f, uint32_t batch) {
  const size_t per = (size_t)f * f * n_prev * n_cur + n_cur;
  const size_t cap = (size_t)256 << 20;  // chunk over samples beyond 256 MiB
  size_t chunk = batch;
  if (chunk * per * sizeof(float) > cap) chunk = cap / (per * sizeof(float));
  if (chunk == 0) chunk = 1;
  return chunk * per * sizeof(float);
}

int conv_grad_acc(const float* in, const float* d, float* gW, float* gB, uint32_t n_prev,
                  uint32_t n_cur, uint32_t f, uint32_t out_w, uint32_t out_h, uint32_t batch,
                  void* ws, size_t ws_bytes, hipStream_t s) {
  const uint32_t nW = f * f * n_prev * n_cur;
  const size_t per = (size_t)nW + n_cur;
  const size_t chunk_max = ws_bytes / (per * sizeof(float));
  if (chunk_max == 0)
    return fail(SRCNN_ERR_WORKSPACE, "conv_grad_acc: workspace %zu B < one sample's partials %zu B",
                ws_bytes, per * sizeof(float));
  float* part = static_cast<float*>(ws);
  for (uint32_t s0 = 0; s0 < batch; s0 += (uint32_t)chunk_max) {
    const uint32_t chunk = (uint32_t)((batch - s0) < chunk_max ? (batch - s0) : chunk_max);
    {
      SRCNN_PROFILE("grad_partial_generic", s);
      hipLaunchKernelGGL(grad_partial_kernel, dim3(grid_for(per * chunk, 256)), dim3(256), 0, s,
                         in, d, part, n_prev, n_cur, f, out_w, out_h, s0, chunk);
      SRCNN_LAUNCH_TRY();
    }
    {
      SRCNN_PROFILE("grad_reduce_generic", s);
      hipLaunchKernelGGL(grad_reduce_kernel, dim3(grid_for(per, 256)), dim3(256), 0, s, part, gW,
                         gB, nW, n_cur, chunk);
      SRCNN_LAUNCH_TRY();
    }
  }
  return SRCNN_OK;
}

}  // namespace generic

// ---------------------------------------------------------------------------
// update: src/kernel/update_parameters.cl:1-33 (shape-free, shared by all paths)
// ---------------------------------------------------------------------------
__global__ void sgd_update_kernel(float* __restrict__ W, float* __restrict__ B,
                                  const float* __restrict__ gW, const float* __restrict__ gB,
                                  float* __restrict__ dW, float* __restrict__ dB, float mu,
                                  float wd, float lr, float batch, uint32_t nW, uint32_t nB) {
  const uint32_t n = nW > nB ? nW : nB;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    if (i < nW) {
      const float w = W[i];
      const float dw = mu * dW[i] + lr * gW[i] + wd * w;
      W[i] = w - dw / batch;
      dW[i] = dw;
    }
    if (i < nB) {
      const float db = mu * dB[i] + lr * gB[i];
      B[i] -= db / batch;
      dB[i] = db;
    }
  }
}

int sgd_update(float* W, float* B, const float* gW, const float* gB, float* dW, float* dB,
               float mu, float wd, float lr, uint32_t batch, uint32_t nW, uint32_t nB,
               hipStream_t s) {
  const uint32_t n = nW > nB ? nW : nB;
  SRCNN_PROFILE("sgd_update", s);
  hipLaunchKernelGGL(sgd_update_kernel, dim3(grid_for(n, 256)), dim3(256), 0, s, W, B, gW, gB,
                     dW, dB, mu, wd, lr, (float)batch, nW, nB);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// All three layers' updates and the gradient zero-fill in one launch over the
// flat [W1|B1|W2|B2|W3|B3] buffers (ConfigBasedDataPipeline.cpp:325-361 runs
// update_params x3 + six zero-fills).  Same arithmetic as sgd_update_kernel per
// element; off[] = the six segment offsets, off[6] = P.
struct UpdateSegs {
  uint32_t off[7];
  float lr[3];
};

__global__ void update_all_kernel(float* __restrict__ P, float* __restrict__ G,
                                  float* __restrict__ M, UpdateSegs sg, float mu, float wd,
                                  float batch) {
  const uint32_t n = sg.off[6];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    int seg = 0;
#pragma unroll
    for (int k = 1; k < 6; k++) seg += i >= sg.off[k];
    // weights: update_parameters.cl:14-24; biases, no weight decay: :26-32
    float w = P[i], m = M[i];
    fused::sgd_step(w, m, seg, G[i], sg.lr[seg >> 1], mu, wd, batch);
    P[i] = w;
    M[i] = m;
    G[i] = 0.0f;
  }
}

int update_all(float* params, float* grads, float* mom, const size_t* off, size_t total,
               const float* lr, float mu, float wd, uint32_t batch, hipStream_t s) {
  UpdateSegs sg;
  for (int k = 0; k < 6; k++) sg.off[k] = (uint32_t)off[k];
  sg.off[6] = (uint32_t)total;
  for (int k = 0; k < 3; k++) sg.lr[k] = lr[k];
  SRCNN_PROFILE("update_all", s);
  hipLaunchKernelGGL(update_all_kernel, dim3(grid_for(total, 256, 2048)), dim3(256), 0, s, params,
                     grads, mom, sg, mu, wd, (float)batch);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// srcnn_train_fwd_bwd_lazy off the fused path: the pending update out of
// place (Po, Mo), then the gradient buffer zeroed for the step's accumulation
__global__ void lazy_update_kernel(fused::LazyUpdate u) {
  float* G = const_cast<float*>(u.G);
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < u.off[6]; i += gridDim.x * blockDim.x) {
    const int seg = fused::param_seg(u.off, i);
    float w = u.P[i], m = u.M[i];
    fused::sgd_step(w, m, seg, G[i], u.lr[seg >> 1], u.mu, u.wd, u.batch);
    u.Po[i] = w;
    u.Mo[i] = m;
    G[i] = 0.0f;
  }
}

int lazy_update(const fused::LazyUpdate& u, hipStream_t s) {
  SRCNN_PROFILE("update_all", s);
  kernels_note("lazy_update");
  hipLaunchKernelGGL(lazy_update_kernel, dim3(grid_for(u.off[6], 256, 2048)), dim3(256), 0, s, u);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

int preload_update() {
  const void* k[] = {(const void*)update_all_kernel, (const void*)lazy_update_kernel};
  return resolve_kernels(k, 2);
}

// ---------------------------------------------------------------------------
// deterministic reductions (sum.cl:35-68, squared_error.cl:36-92):
// pass 1: fixed grid, per-block tree in LDS -> partial[block]
// pass 2: one block reduces the partials in fixed order
// ---------------------------------------------------------------------------
constexpr uint32_t kReduceBlock = 256;
constexpr uint32_t kReduceMaxBlocks = 1024;

uint32_t reduce_blocks(size_t len) {
  return grid_for(len, kReduceBlock * 8, kReduceMaxBlocks);
}

__device__ inline float block_sum(float v, float* lds) {
  // wavefront (64-lane) shuffle tree, then across the block's 4 waves
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (lane == 0) lds[wave] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.0f;
    for (int w = 0; w < (int)(blockDim.x >> 6); w++) t += lds[w];
    lds[0] = t;
  }
  __syncthreads();
  return lds[0];
}

template <int MODE>  // 0 sum, 1 sum of squares, 2 squared error
__global__ void reduce_partial_kernel(const float* __restrict__ a, const float* __restrict__ gt,
                                      float* __restrict__ part, size_t len, uint32_t gt_w,
                                      uint32_t gt_h, uint32_t out_w, uint32_t out_h) {
  __shared__ float lds[16];
  const uint32_t pad = MODE == 2 ? (gt_w - out_w) / 2 : 0;
  float acc = 0.0f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < len;
       i += (size_t)gridDim.x * blockDim.x) {
    float v = a[i];
    if (MODE == 1) v = v * v;
    if (MODE == 2) {
      const uint32_t c = i % out_w;
      const size_t t = i / out_w;
      const uint32_t r = t % out_h;
      const size_t smp = t / out_h;
      const float d = v - gt[smp * gt_w * gt_h + (size_t)(r + pad) * gt_w + pad + c];
      v = d * d;
    }
    acc += v;
  }
  acc = block_sum(acc, lds);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

// MODE_OUT 0: *out = sum ; 1: *out += sum ; 2: mean -> *out and data -= mean
__global__ void reduce_final_kernel(const float* __restrict__ part, uint32_t nparts,
                                    float* __restrict__ out, int accumulate) {
  __shared__ float lds[16];
  float acc = 0.0f;
  for (uint32_t i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  acc = block_sum(acc, lds);
  if (threadIdx.x == 0) *out = accumulate ? *out + acc : acc;
}

int reduce(int mode, const float* a, const float* gt, size_t len, uint32_t gt_w, uint32_t gt_h,
           uint32_t out_w, uint32_t out_h, float* result, int accumulate, void* ws,
           size_t ws_bytes, hipStream_t s) {
  const uint32_t nb = reduce_blocks(len);
  if (ws_bytes < nb * sizeof(float))
    return fail(SRCNN_ERR_WORKSPACE, "reduction: workspace %zu B < %zu B", ws_bytes,
                nb * sizeof(float));
  float* part = static_cast<float*>(ws);
  SRCNN_PROFILE(mode == 2 ? "sq_err" : "sum", s);
  if (mode == 0)
    hipLaunchKernelGGL(reduce_partial_kernel<0>, dim3(nb), dim3(kReduceBlock), 0, s, a, gt, part,
                       len, gt_w, gt_h, out_w, out_h);
  else if (mode == 1)
    hipLaunchKernelGGL(reduce_partial_kernel<1>, dim3(nb), dim3(kReduceBlock), 0, s, a, gt, part,
                       len, gt_w, gt_h, out_w, out_h);
  else
    hipLaunchKernelGGL(reduce_partial_kernel<2>, dim3(nb), dim3(kReduceBlock), 0, s, a, gt, part,
                       len, gt_w, gt_h, out_w, out_h);
  SRCNN_LAUNCH_TRY();
  hipLaunchKernelGGL(reduce_final_kernel, dim3(1), dim3(kReduceBlock), 0, s, part, nb, result,
                     accumulate);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

__global__ void sub_scalar_kernel(float* __restrict__ d, float v, size_t len) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < len;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = d[i] - v;
}

__global__ void sub_mean_kernel(float* __restrict__ d, const float* __restrict__ sum,
                                float* __restrict__ mean_out, size_t len) {
  const float m = *sum / (float)len;  // DataPipeline.cpp:275
  if (mean_out && blockIdx.x == 0 && threadIdx.x == 0) *mean_out = m;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < len;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = d[i] - m;
}

__global__ void fill_kernel(float* __restrict__ d, float v, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x)
    d[i] = v;
}

int fill(float* d, float v, size_t n, hipStream_t s) {
  if (n == 0) return SRCNN_OK;
  SRCNN_PROFILE("fill", s);
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for(n, 256, 4096)), dim3(256), 0, s, d, v, n);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

// ---------------------------------------------------------------------------
// luma: extract_luma.cl:7-23, swap_luma.cl:18-69 (image2d -> plain RGBA8 buffer)
// ---------------------------------------------------------------------------
__global__ void extract_luma_kernel(const uint8_t* __restrict__ rgba, float* __restrict__ luma,
                                    uint32_t n, int normalize) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uchar4 p = reinterpret_cast<const uchar4*>(rgba)[i];
    const float v = (float)p.x * 0.299f + (float)p.y * 0.587f + (float)p.z * 0.114f;
    luma[i] = normalize ? v / 255.0f : v;
  }
}

__global__ void swap_luma_kernel(const uint8_t* __restrict__ rgba, const float* __restrict__ nl,
                                 uint8_t* __restrict__ rgb, uint32_t w, uint32_t h,
                                 uint32_t lw, uint32_t lh) {
  const int pad = (int)(w - lw) / 2;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < w * h; i += gridDim.x * blockDim.x) {
    const int x = i % w, y = i / w;
    const int lx = x - pad, ly = y - pad;
    const uchar4 p = reinterpret_cast<const uchar4*>(rgba)[i];
    unsigned c0 = p.x, c1 = p.y, c2 = p.z;
    if (!(lx < 0 || lx >= (int)lw || ly < 0 || ly >= (int)lh)) {
      const float r = p.x, g = p.y, b = p.z;
      const float Y = nl[(size_t)ly * lw + lx] * 255.0f;
      const float Cb = r * -0.1687f + g * -0.3312f + b * 0.5f;
      const float Cr = r * 0.5f + g * -0.4186f + b * -0.0813f;
      const float R = fminf(fmaxf(Y * 1.0f + Cb * 0.0f + Cr * 1.4f, 0.0f), 255.0f);
      const float G = fminf(fmaxf(Y * 1.0f + Cb * -0.343f + Cr * -0.711f, 0.0f), 255.0f);
      const float Bc = fminf(fmaxf(Y * 1.0f + Cb * 1.765f + Cr * 0.0f, 0.0f), 255.0f);
      c0 = (unsigned)R;
      c1 = (unsigned)G;
      c2 = (unsigned)Bc;
    }
    rgb[3 * (size_t)i + 0] = (uint8_t)c0;
    rgb[3 * (size_t)i + 1] = (uint8_t)c1;
    rgb[3 * (size_t)i + 2] = (uint8_t)c2;
  }
}

int extract_luma(const uint8_t* rgba, float* luma, uint32_t w, uint32_t h, int normalize,
                 hipStream_t s) {
  SRCNN_PROFILE("extract_luma", s);
  hipLaunchKernelGGL(extract_luma_kernel, dim3(grid_for((size_t)w * h, 256)), dim3(256), 0, s,
                     rgba, luma, w * h, normalize);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

int swap_luma(const uint8_t* rgba, const float* nl, uint8_t* rgb, uint32_t w, uint32_t h,
              uint32_t lw, uint32_t lh, hipStream_t s) {
  SRCNN_PROFILE("swap_luma", s);
  hipLaunchKernelGGL(swap_luma_kernel, dim3(grid_for((size_t)w * h, 256)), dim3(256), 0, s, rgba,
                     nl, rgb, w, h, lw, lh);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

int sub_scalar(float* d, float v, size_t len, hipStream_t s) {
  if (len == 0) return SRCNN_OK;
  SRCNN_PROFILE("sub_from_all", s);
  hipLaunchKernelGGL(sub_scalar_kernel, dim3(grid_for(len, 256, 4096)), dim3(256), 0, s, d, v, len);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

int sub_mean(float* d, size_t len, float* mean_out, void* ws, size_t ws_bytes, hipStream_t s) {
  const uint32_t nb = reduce_blocks(len);
  if (ws_bytes < (nb + 1) * sizeof(float))
    return fail(SRCNN_ERR_WORKSPACE, "sub_mean: workspace %zu B < %zu B", ws_bytes,
                (nb + 1) * sizeof(float));
  float* sum = static_cast<float*>(ws) + nb;
  int rc = reduce(0, d, nullptr, len, 0, 0, 0, 0, sum, 0, ws, ws_bytes, s);
  if (rc) return rc;
  SRCNN_PROFILE("sub_mean", s);
  hipLaunchKernelGGL(sub_mean_kernel, dim3(grid_for(len, 256, 4096)), dim3(256), 0, s, d, sum,
                     mean_out, len);
  SRCNN_LAUNCH_TRY();
  return SRCNN_OK;
}

}  // namespace srcnn
