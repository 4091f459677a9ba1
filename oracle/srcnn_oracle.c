/*
 * srcnn_oracle.c -- CPU restatement of the reference SRCNN hot path.
 *
 * TEST INFRASTRUCTURE ONLY (see srcnn_oracle.h).  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this.
 *
 * Each routine cites the reference file:line it restates.  Loop nests keep
 * the reference's per-work-item float accumulation order; outer loops are
 * reordered only where that leaves every accumulator's order unchanged
 * (noted inline).  OpenMP parallelises over samples (and over output rows
 * in forward / deltas), which never shares an accumulator between threads.
 */
#include "srcnn_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

int oracle_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

/* ------------------------------------------------------------------ */
/* forward: src/kernel/layer_uber_kernel.cl:36-96                       */
/* ------------------------------------------------------------------ */
void oracle_conv_fwd(const float* in, float* out, const float* W,
                     const float* B, int in_w, int in_h, int n_prev,
                     int n_cur, int f, int relu, int batch) {
  const int out_w = in_w - f + 1, out_h = in_h - f + 1;  /* :48-49 */
  /* One work item per output pixel (:43-56); the OpenMP team splits the
   * (sample, row) pairs, so a single large frame (batch 1) uses every core
   * and every accumulator keeps the reference's tap order. */
#pragma omp parallel
  {
    float* vals = (float*)malloc(sizeof(float) * (size_t)n_cur);
#pragma omp for collapse(2) schedule(static)
    for (int s = 0; s < batch; s++) {
      for (int y = 0; y < out_h; y++) {
        const float* img = in + (size_t)s * n_prev * in_w * in_h;    /* :51 */
        float* dst = out + (size_t)s * n_cur * out_w * out_h;        /* :52 */
        for (int x = 0; x < out_w; x++) {
          for (int n = 0; n < n_cur; n++) vals[n] = 0.0f;            /* :59-62 */
          for (int dy = 0; dy < f; dy++) {                           /* :70 */
            for (int dx = 0; dx < f; dx++) {                         /* :71 */
              const float* px = img + ((size_t)(y + dy) * in_w + (x + dx)) * n_prev;
              const float* w2d = W + (size_t)(dy * f + dx) * n_cur * n_prev;
              for (int k = 0; k < n_prev; k++) {                     /* :76 */
                const float v = px[k];
                const float* w3d = w2d + (size_t)k * n_cur;
                for (int n = 0; n < n_cur; n++) vals[n] += w3d[n] * v; /* :80-82 */
              }
            }
          }
          float* o = dst + ((size_t)y * out_w + x) * n_cur;          /* :56 */
          for (int n = 0; n < n_cur; n++) {                          /* :88-95 */
            const float r = vals[n] + B[n];
            o[n] = relu ? fmaxf(r, 0.0f) : r;
          }
        }
      }
    }
    free(vals);
  }
}

/* ------------------------------------------------------------------ */
/* last layer delta: src/kernel/last_layer_delta.cl:14-50               */
/* ------------------------------------------------------------------ */
void oracle_last_delta(const float* gt, const float* y, float* d, int gt_w,
                       int gt_h, int out_w, int out_h, int batch) {
  const int padding = (gt_w - out_w) / 2;                          /* :25 */
  for (int s = 0; s < batch; s++) {
    const float* g = gt + (size_t)s * gt_w * gt_h;                 /* :27 */
    const float* a = y + (size_t)s * out_w * out_h;                /* :28 */
    float* o = d + (size_t)s * out_w * out_h;
    for (int r = 0; r < out_h; r++)
      for (int c = 0; c < out_w; c++) {
        const float t = g[(size_t)(r + padding) * gt_w + padding + c]; /* :34-35 */
        const float v = a[(size_t)r * out_w + c];
        const float diff = v - t;                                  /* :42 */
        const float relu_deriv = v > 0.0f ? 1.0f : 0.0f;           /* :45 quirk */
        o[(size_t)r * out_w + c] = diff * relu_deriv;              /* :48 */
      }
  }
}

/* ------------------------------------------------------------------ */
/* deltas: src/kernel/layer_deltas.cl:42-127                            */
/* ------------------------------------------------------------------ */
/* mask == NULL: relu' = [y_curr > 0] as in the reference (:72-77); else
 * relu' = mask[same index] (the masked-oracle entry point below) */
static void conv_delta_impl(const float* d_next, const float* y_curr,
                            const uint8_t* mask, float* d_curr,
                            const float* W_next, int f_next, int n_curr,
                            int n_next, int curr_w, int curr_h, int batch) {
  const int next_w = curr_w - f_next + 1, next_h = curr_h - f_next + 1; /* :56-57 */
  /* (sample, row) pairs split over the OpenMP team, as in oracle_conv_fwd */
#pragma omp parallel
  {
    float* acc = (float*)malloc(sizeof(float) * (size_t)n_curr);
    float* deriv = (float*)malloc(sizeof(float) * (size_t)n_curr);
#pragma omp for collapse(2) schedule(static)
    for (int s = 0; s < batch; s++) {
      for (int y = 0; y < curr_h; y++) {
        const float* yc = y_curr + (size_t)s * n_curr * curr_w * curr_h;  /* :59-60 */
        const float* dn = d_next + (size_t)s * n_next * next_w * next_h;  /* :61-62 */
        float* dc = d_curr + (size_t)s * n_curr * curr_w * curr_h;
        for (int x = 0; x < curr_w; x++) {
          const size_t idx = ((size_t)y * curr_w + x) * n_curr;        /* :55 */
          for (int n = 0; n < n_curr; n++) {                           /* :72-77 */
            acc[n] = 0.0f;
            deriv[n] = (mask ? mask[(size_t)s * n_curr * curr_w * curr_h + idx + n] != 0
                             : yc[idx + n] > 0.0f) ? 1.0f : 0.0f;
          }
          for (int dy = 0; dy < f_next; dy++) {                        /* :79 */
            for (int dx = 0; dx < f_next; dx++) {                      /* :80 */
              const int nx = x - dx, ny = y - dy;                      /* :82 */
              const int in_range = nx >= 0 && nx < next_w && ny >= 0 && ny < next_h; /* :94-96 */
              /* out-of-range terms add (0*w)*deriv == 0: skipping them
               * leaves every accumulator unchanged. */
              if (!in_range) continue;
              const size_t w2d = (size_t)(dy * f_next + dx) * n_next * n_curr; /* :83-84 */
              const float* dptr = dn + ((size_t)ny * next_w + nx) * n_next;     /* :91-93 */
              for (int k = 0; k < n_next; k++) {                       /* :86 */
                const float delta = dptr[k];                           /* :97-100 */
                for (int n = 0; n < n_curr; n++) {                     /* :102 */
                  const float w = W_next[w2d + (size_t)n * n_next + k]; /* :105-106 */
                  acc[n] += delta * w * deriv[n];                      /* :112 */
                }
              }
            }
          }
          for (int n = 0; n < n_curr; n++) dc[idx + n] = acc[n];       /* :121-123 */
        }
      }
    }
    free(acc);
    free(deriv);
  }
}

void oracle_conv_delta(const float* d_next, const float* y_curr,
                       float* d_curr, const float* W_next, int f_next,
                       int n_curr, int n_next, int curr_w, int curr_h,
                       int batch) {
  conv_delta_impl(d_next, y_curr, NULL, d_curr, W_next, f_next, n_curr, n_next,
                  curr_w, curr_h, batch);
}

/* ------------------------------------------------------------------ */
/* gradients: src/kernel/backpropagate.cl:56-114                        */
/* ------------------------------------------------------------------ */
void oracle_conv_grad_acc(const float* in, const float* delta, float* gW,
                          float* gB, int n_prev, int n_cur, int f, int out_w,
                          int out_h, int batch) {
  const int in_w = out_w + f - 1, in_h = out_h + f - 1;             /* :66-67 */
  const size_t nW = (size_t)f * f * n_prev * n_cur;                  /* :69-71 */
  const size_t per = nW + (size_t)n_cur;
  float* part = (float*)calloc((size_t)batch * per, sizeof(float));
#pragma omp parallel for schedule(static)
  for (int s = 0; s < batch; s++) {
    /* One work-item per (weight id, sample) sums over all output pixels
     * in (row, col) order (:89-106).  Visiting pixels in the outer loop
     * and weights in the inner loop keeps each weight's order intact. */
    float* gw = part + (size_t)s * per;
    float* gb = gw + nW;
    const float* img = in + (size_t)s * n_prev * in_w * in_h;        /* :75 */
    const float* dl = delta + (size_t)s * n_cur * out_w * out_h;     /* :73-74 */
    for (int row = 0; row < out_h; row++) {
      for (int col = 0; col < out_w; col++) {
        const float* dp = dl + ((size_t)row * out_w + col) * n_cur;  /* :92-93 */
        for (int n = 0; n < n_cur; n++) gb[n] += dp[n];              /* :94 */
        for (int dy = 0; dy < f; dy++) {
          for (int dx = 0; dx < f; dx++) {
            const float* ip = img + ((size_t)(row + dy) * in_w + (col + dx)) * n_prev; /* :99-103 */
            float* w2 = gw + (size_t)(dy * f + dx) * n_prev * n_cur;
            for (int k = 0; k < n_prev; k++) {
              const float v = ip[k];
              float* w3 = w2 + (size_t)k * n_cur;                    /* id decode :78-85 */
              for (int n = 0; n < n_cur; n++) w3[n] += v * dp[n];    /* :104 */
            }
          }
        }
      }
    }
  }
  /* :110-112, race-free: per-sample sums added in sample order. */
  for (int s = 0; s < batch; s++) {
    const float* gw = part + (size_t)s * per;
    for (size_t i = 0; i < nW; i++) gW[i] += gw[i];
    for (int n = 0; n < n_cur; n++) gB[n] += gw[nW + n];
  }
  free(part);
}

/* ------------------------------------------------------------------ */
/* update: src/kernel/update_parameters.cl:1-33                         */
/* ------------------------------------------------------------------ */
void oracle_sgd_update(float* W, float* B, const float* gW, const float* gB,
                       float* dW_prev, float* dB_prev, float momentum,
                       float wd, float lr, unsigned batch, int nW, int nB) {
  for (int i = 0; i < nW; i++) {                                     /* :17-24 */
    const float w = W[i];
    const float dw = momentum * dW_prev[i] + lr * gW[i] + wd * w;    /* :19-21 */
    W[i] = w - dw / (float)batch;                                    /* :22 */
    dW_prev[i] = dw;                                                 /* :23 */
  }
  for (int i = 0; i < nB; i++) {                                     /* :27-32 */
    const float db = momentum * dB_prev[i] + lr * gB[i];             /* :28-29 */
    B[i] -= db / (float)batch;                                       /* :30 */
    dB_prev[i] = db;                                                 /* :31 */
  }
}

/* ------------------------------------------------------------------ */
/* squared error: src/kernel/squared_error.cl:36-92 (sum in double, the */
/* reference's order is non-deterministic)                               */
/* ------------------------------------------------------------------ */
float oracle_sq_err(const float* gt, const float* y, int gt_w, int gt_h,
                    int out_w, int out_h, int batch) {
  const int padding = (gt_w - out_w) / 2;                            /* :48 */
  double acc = 0.0;
  for (int s = 0; s < batch; s++) {
    const float* g = gt + (size_t)s * gt_w * gt_h;
    const float* a = y + (size_t)s * out_w * out_h;
    for (int r = 0; r < out_h; r++)
      for (int c = 0; c < out_w; c++) {
        const float t = g[(size_t)(r + padding) * gt_w + padding + c]; /* :60-61 */
        const float d = a[(size_t)r * out_w + c] - t;                /* :68 */
        acc += (double)(d * d);                                      /* :69 */
      }
  }
  return (float)acc;
}

/* sum.cl:35-68 (LDS tree + CAS atomic -> order non-deterministic; the
 * oracle sums in double). */
float oracle_sum(const float* data, size_t len, int squared) {
  double acc = 0.0;
  for (size_t i = 0; i < len; i++) {
    float v = data[i];
    if (squared) v = v * v;                                          /* :44-46 */
    acc += v;
  }
  return (float)acc;
}

/* subtract_from_all.cl:1-8 */
void oracle_sub_from_all(float* data, float value, size_t len) {
  for (size_t i = 0; i < len; i++) data[i] = data[i] - value;
}

/* extract_luma.cl:5-22: dot(rgba, {0.299, 0.587, 0.114, 0}) (/255) */
void oracle_extract_luma(const uint8_t* rgba, float* luma, int w, int h,
                         int normalize) {
  for (int i = 0; i < w * h; i++) {
    const float r = rgba[4 * i + 0], g = rgba[4 * i + 1], b = rgba[4 * i + 2];
    const float v = r * 0.299f + g * 0.587f + b * 0.114f;
    luma[i] = normalize ? v / 255.0f : v;                            /* :17-21 */
  }
}

/* swap_luma.cl:7-68 */
void oracle_swap_luma(const uint8_t* rgba, const float* new_luma,
                      uint8_t* rgb, int w, int h, int luma_w, int luma_h) {
  const int padding = (w - luma_w) / 2;                              /* :24 */
  for (int y = 0; y < h; y++)
    for (int x = 0; x < w; x++) {
      const int lx = x - padding, ly = y - padding;                  /* :26 */
      const size_t idx = (size_t)y * w + x;
      const uint8_t* p = rgba + 4 * idx;
      unsigned c0, c1, c2;
      if (lx < 0 || lx >= luma_w || ly < 0 || ly >= luma_h) {        /* :37-42 */
        c0 = p[0];
        c1 = p[1];
        c2 = p[2];
      } else {
        const float r = p[0], g = p[1], b = p[2];
        const float Y = new_luma[(size_t)ly * luma_w + lx] * 255.0f; /* :49-50 */
        const float Cb = r * -0.1687f + g * -0.3312f + b * 0.5f;     /* :8, :51 */
        const float Cr = r * 0.5f + g * -0.4186f + b * -0.0813f;     /* :9, :52 */
        float R = Y * 1.0f + Cb * 0.0f + Cr * 1.4f;                  /* :13, :54 */
        float G = Y * 1.0f + Cb * -0.343f + Cr * -0.711f;            /* :14, :55 */
        float Bc = Y * 1.0f + Cb * 1.765f + Cr * 0.0f;               /* :15, :56 */
        R = fminf(fmaxf(R, 0.0f), 255.0f);                           /* :57 */
        G = fminf(fmaxf(G, 0.0f), 255.0f);
        Bc = fminf(fmaxf(Bc, 0.0f), 255.0f);
        c0 = (unsigned)R;                                            /* :60-62 rtz */
        c1 = (unsigned)G;
        c2 = (unsigned)Bc;
      }
      rgb[3 * idx + 0] = (uint8_t)c0;                                /* :66-68 */
      rgb[3 * idx + 1] = (uint8_t)c1;
      rgb[3 * idx + 2] = (uint8_t)c2;
    }
}

/* ------------------------------------------------------------------ */
/* orchestration: src/ConfigBasedDataPipeline.cpp                        */
/* ------------------------------------------------------------------ */
size_t oracle_param_count(int n1, int n2, int f1, int f2, int f3) {
  return (size_t)f1 * f1 * 1 * n1 + n1 + (size_t)f2 * f2 * n1 * n2 + n2 +
         (size_t)f3 * f3 * n2 * 1 + 1;
}

/* LayerData(1,n1,f1), (n1,n2,f2), (n2,1,f3): ConfigBasedDataPipeline.cpp:27-29 */
static void layer_offsets(int n1, int n2, int f1, int f2, int f3,
                          size_t off[6]) {
  off[0] = 0;                                   /* W1 */
  off[1] = off[0] + (size_t)f1 * f1 * n1;       /* B1 */
  off[2] = off[1] + (size_t)n1;                 /* W2 */
  off[3] = off[2] + (size_t)f2 * f2 * n1 * n2;  /* B2 */
  off[4] = off[3] + (size_t)n2;                 /* W3 */
  off[5] = off[4] + (size_t)f3 * f3 * n2;       /* B3 */
}

size_t oracle_train_acts_floats(int n1, int n2, int f1, int f2, int f3,
                                int w, int h, int batch) {
  const size_t o1 = (size_t)(w - f1 + 1) * (h - f1 + 1);
  const size_t o2 = (size_t)(w - f1 - f2 + 2) * (h - f1 - f2 + 2);
  const size_t o3 = (size_t)(w - f1 - f2 - f3 + 3) * (h - f1 - f2 - f3 + 3);
  /* A1, A2, A3, D3, D2, D1 (ConfigBasedDataPipeline.cpp:82-108) */
  return (size_t)batch * (2 * o1 * n1 + 2 * o2 * n2 + 2 * o3);
}

void oracle_train_fwd_bwd(int n1, int n2, int f1, int f2, int f3,
                          const float* X, const float* T, int w, int h,
                          int batch, const float* params, float* grads,
                          float* acts) {
  size_t off[6];
  layer_offsets(n1, n2, f1, f2, f3, off);
  const int w1 = w - f1 + 1, h1 = h - f1 + 1;
  const int w2 = w1 - f2 + 1, h2 = h1 - f2 + 1;
  const int w3 = w2 - f3 + 1, h3 = h2 - f3 + 1;
  const size_t s1 = (size_t)batch * w1 * h1 * n1;
  const size_t s2 = (size_t)batch * w2 * h2 * n2;
  const size_t s3 = (size_t)batch * w3 * h3;
  float* buf = acts ? acts
                    : (float*)malloc(sizeof(float) *
                                     oracle_train_acts_floats(n1, n2, f1, f2, f3, w, h, batch));
  float *A1 = buf, *A2 = A1 + s1, *A3 = A2 + s2, *D3 = A3 + s3, *D2 = D3 + s3,
        *D1 = D2 + s2;
  /* forward, ConfigBasedDataPipeline.cpp:200-241 */
  oracle_conv_fwd(X, A1, params + off[0], params + off[1], w, h, 1, n1, f1, 1, batch);
  oracle_conv_fwd(A1, A2, params + off[2], params + off[3], w1, h1, n1, n2, f2, 1, batch);
  oracle_conv_fwd(A2, A3, params + off[4], params + off[5], w2, h2, n2, 1, f3, 0, batch);
  /* backward, ConfigBasedDataPipeline.cpp:243-323 */
  oracle_last_delta(T, A3, D3, w, h, w3, h3, batch);
  oracle_conv_delta(D3, A2, D2, params + off[4], f3, n2, 1, w2, h2, batch);
  oracle_conv_delta(D2, A1, D1, params + off[2], f2, n1, n2, w1, h1, batch);
  oracle_conv_grad_acc(A2, D3, grads + off[4], grads + off[5], n2, 1, f3, w3, h3, batch);
  oracle_conv_grad_acc(A1, D2, grads + off[2], grads + off[3], n1, n2, f2, w2, h2, batch);
  oracle_conv_grad_acc(X, D1, grads + off[0], grads + off[1], 1, n1, f1, w1, h1, batch);
  if (!acts) free(buf);
}

/* oracle_train_fwd_bwd with the ReLU decisions taken from outside:
 * A1 = m1 ? pre1 : 0 (layer_uber_kernel.cl:88-95 with the comparison
 * replaced), relu'(A1) = m1, likewise m2 for layer 2 (layer_deltas.cl:72-77),
 * and m3 for the last layer's relu' quirk (last_layer_delta.cl:45).  m1 / m2 /
 * m3 are [batch][h1][w1][n1] / [batch][h2][w2][n2] / [batch][h3][w3] bytes
 * (0 / 1).  With the f64 build and the HIP path's own activation signs as the
 * masks, the result is the exact gradient of the decisions the HIP path made:
 * the parity tests use it to separate ReLU-decision flips (a pre-activation
 * within fp32 rounding of zero) from accumulation error. */
void oracle_train_fwd_bwd_masked(int n1, int n2, int f1, int f2, int f3,
                                 const float* X, const float* T, int w, int h,
                                 int batch, const float* params, float* grads,
                                 float* acts, const uint8_t* m1,
                                 const uint8_t* m2, const uint8_t* m3) {
  size_t off[6];
  layer_offsets(n1, n2, f1, f2, f3, off);
  const int w1 = w - f1 + 1, h1 = h - f1 + 1;
  const int w2 = w1 - f2 + 1, h2 = h1 - f2 + 1;
  const int w3 = w2 - f3 + 1, h3 = h2 - f3 + 1;
  const size_t s1 = (size_t)batch * w1 * h1 * n1;
  const size_t s2 = (size_t)batch * w2 * h2 * n2;
  const size_t s3 = (size_t)batch * w3 * h3;
  float* buf = acts ? acts
                    : (float*)malloc(sizeof(float) *
                                     oracle_train_acts_floats(n1, n2, f1, f2, f3, w, h, batch));
  float *A1 = buf, *A2 = A1 + s1, *A3 = A2 + s2, *D3 = A3 + s3, *D2 = D3 + s3,
        *D1 = D2 + s2;
  oracle_conv_fwd(X, A1, params + off[0], params + off[1], w, h, 1, n1, f1, 0, batch);
  for (size_t i = 0; i < s1; i++) A1[i] = m1[i] ? A1[i] : 0.0f;
  oracle_conv_fwd(A1, A2, params + off[2], params + off[3], w1, h1, n1, n2, f2, 0, batch);
  for (size_t i = 0; i < s2; i++) A2[i] = m2[i] ? A2[i] : 0.0f;
  oracle_conv_fwd(A2, A3, params + off[4], params + off[5], w2, h2, n2, 1, f3, 0, batch);
  oracle_last_delta(T, A3, D3, w, h, w3, h3, batch);
  for (size_t i = 0; i < s3; i++) /* last_layer_delta.cl:42-48 with relu' = m3 */
    if (m3[i] != (A3[i] > 0.0f)) {
      const size_t s = i / ((size_t)w3 * h3), r = i % ((size_t)w3 * h3);
      const int pad = (w - w3) / 2;
      const float t = T[s * (size_t)w * h + (r / w3 + pad) * (size_t)w + pad + r % w3];
      D3[i] = m3[i] ? A3[i] - t : 0.0f;
    }
  conv_delta_impl(D3, A2, m2, D2, params + off[4], f3, n2, 1, w2, h2, batch);
  conv_delta_impl(D2, A1, m1, D1, params + off[2], f2, n1, n2, w1, h1, batch);
  oracle_conv_grad_acc(A2, D3, grads + off[4], grads + off[5], n2, 1, f3, w3, h3, batch);
  oracle_conv_grad_acc(A1, D2, grads + off[2], grads + off[3], n1, n2, f2, w2, h2, batch);
  oracle_conv_grad_acc(X, D1, grads + off[0], grads + off[1], 1, n1, f1, w1, h1, batch);
  if (!acts) free(buf);
}

void oracle_update_all(int n1, int n2, int f1, int f2, int f3, float* params,
                       float* grads, float* momentum_bufs, float momentum,
                       float wd, const float* lr, unsigned batch) {
  size_t off[6];
  layer_offsets(n1, n2, f1, f2, f3, off);
  const size_t total = oracle_param_count(n1, n2, f1, f2, f3);
  /* layer 3, 2, 1 order: ConfigBasedDataPipeline.cpp:325-361 */
  for (int l = 2; l >= 0; l--) {
    const size_t wo = off[2 * l], bo = off[2 * l + 1];
    const size_t nW = bo - wo;
    const size_t nB = (l == 2 ? total : off[2 * l + 2]) - bo;
    oracle_sgd_update(params + wo, params + bo, grads + wo, grads + bo,
                      momentum_bufs + wo, momentum_bufs + bo, momentum, wd,
                      lr[l], batch, (int)nW, (int)nB);
  }
  memset(grads, 0, sizeof(float) * total);                           /* :512-517 */
}

void oracle_forward(int n1, int n2, int f1, int f2, int f3, const float* X,
                    int w, int h, int batch, const float* params, float* out) {
  size_t off[6];
  layer_offsets(n1, n2, f1, f2, f3, off);
  const int w1 = w - f1 + 1, h1 = h - f1 + 1;
  const int w2 = w1 - f2 + 1, h2 = h1 - f2 + 1;
  float* A1 = (float*)malloc(sizeof(float) * (size_t)batch * w1 * h1 * n1);
  float* A2 = (float*)malloc(sizeof(float) * (size_t)batch * w2 * h2 * n2);
  oracle_conv_fwd(X, A1, params + off[0], params + off[1], w, h, 1, n1, f1, 1, batch);
  oracle_conv_fwd(A1, A2, params + off[2], params + off[3], w1, h1, n1, n2, f2, 1, batch);
  oracle_conv_fwd(A2, out, params + off[4], params + off[5], w2, h2, n2, 1, f3, 0, batch);
  free(A1);
  free(A2);
}
