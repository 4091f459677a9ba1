/*
 * srcnn_oracle.h -- CPU restatement of the reference SRCNN hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This oracle is the parity checker for the HIP
 * path (tests/, __graft_entry__.smoke()) and the CPU baseline leg of
 * bench.py.  Nothing in the product path (libsrcnn_hip.so, the cnn_sr C++
 * API, the cnn CLI) may link, load or call it.
 *
 * Every function restates one OpenCL kernel of Scthe/cnn-Super-Resolution
 * (src/kernel/NAME.cl) or one orchestration routine of
 * src/ConfigBasedDataPipeline.cpp, with the same loop order, the same
 * layouts and the same quirks.  The only intended divergence is the weight
 * gradient: the reference sums per-sample gradients with a racy
 * non-atomic `+=` (backpropagate.cl:110); the oracle sums them race-free in
 * sample order (the mathematically intended result).
 *
 * Layouts (reference):
 *   activations  per-sample HWC, idx = s*C*W*H + (y*W + x)*C + c
 *                (layer_uber_kernel.cl:51-56)
 *   weights      W[dy][dx][c_in][c_out], c_out innermost
 *                (layer_uber_kernel.cl:3-13)
 *
 * Parity pins: tests/golden/ (fixtures taken from the reference's own
 * test specs and test/data files) -- see tests/test_oracle_golden.py.
 */
#ifndef SRCNN_ORACLE_H
#define SRCNN_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* OpenMP thread count for the CPU-baseline timing; returns the count in use */
int oracle_set_threads(int n);

/* forward conv + bias (+ReLU): layer_uber_kernel.cl:36-96 */
void oracle_conv_fwd(const float* in, float* out, const float* W,
                     const float* B, int in_w, int in_h, int n_prev,
                     int n_cur, int f, int relu, int batch);

/* last-layer delta (quirk: relu' on a linear output): last_layer_delta.cl:14-50 */
void oracle_last_delta(const float* gt, const float* y, float* d, int gt_w,
                       int gt_h, int out_w, int out_h, int batch);

/* delta backprop through the next layer's weights: layer_deltas.cl:42-127.
 * d_curr, y_curr: [batch][curr_h][curr_w][n_curr]
 * d_next:         [batch][curr_h-f_next+1][curr_w-f_next+1][n_next]      */
void oracle_conv_delta(const float* d_next, const float* y_curr,
                       float* d_curr, const float* W_next, int f_next,
                       int n_curr, int n_next, int curr_w, int curr_h,
                       int batch);

/* weight/bias gradient accumulate: backpropagate.cl:56-114 (race-free) */
void oracle_conv_grad_acc(const float* in, const float* delta, float* gW,
                          float* gB, int n_prev, int n_cur, int f, int out_w,
                          int out_h, int batch);

/* momentum SGD + weight decay: update_parameters.cl:1-33 */
void oracle_sgd_update(float* W, float* B, const float* gW, const float* gB,
                       float* dW_prev, float* dB_prev, float momentum,
                       float wd, float lr, unsigned batch, int nW, int nB);

/* sum of squared error over the centre crop: squared_error.cl:36-92 */
float oracle_sq_err(const float* gt, const float* y, int gt_w, int gt_h,
                    int out_w, int out_h, int batch);

/* buffer sum (optionally squared): sum.cl:35-68 */
float oracle_sum(const float* data, size_t len, int squared);

/* data[i] -= value: subtract_from_all.cl:1-8 */
void oracle_sub_from_all(float* data, float value, size_t len);

/* RGBA8 -> luma: extract_luma.cl:7-23 */
void oracle_extract_luma(const uint8_t* rgba, float* luma, int w, int h,
                         int normalize);

/* new luma + original chroma -> RGB8: swap_luma.cl:18-69 */
void oracle_swap_luma(const uint8_t* rgba, const float* new_luma,
                      uint8_t* rgb, int w, int h, int luma_w, int luma_h);

/* One reference training chunk: forward L1..L3, last delta, deltas, grads
 * (ConfigBasedDataPipeline.cpp:200-323).  Parameters/grads use the flat
 * layout [W1|B1|W2|B2|W3|B3].  Grads are ACCUMULATED (+=).  Scratch
 * activations are returned in `acts` if non-NULL (A1|A2|A3|D3|D2|D1 per
 * batch, see oracle_train_acts_floats). */
size_t oracle_param_count(int n1, int n2, int f1, int f2, int f3);
size_t oracle_train_acts_floats(int n1, int n2, int f1, int f2, int f3,
                                int w, int h, int batch);
void oracle_train_fwd_bwd(int n1, int n2, int f1, int f2, int f3,
                          const float* X, const float* T, int w, int h,
                          int batch, const float* params, float* grads,
                          float* acts);

/* the same chunk with the ReLU decisions of layers 1 / 2 / 3 supplied as byte
 * masks (m1: A1's layout, m2: A2's, m3: A3's), for separating ReLU-decision flips from
 * accumulation error in the parity tests (see srcnn_oracle.c) */
void oracle_train_fwd_bwd_masked(int n1, int n2, int f1, int f2, int f3,
                                 const float* X, const float* T, int w, int h,
                                 int batch, const float* params, float* grads,
                                 float* acts, const uint8_t* m1,
                                 const uint8_t* m2, const uint8_t* m3);

/* update all three layers, ConfigBasedDataPipeline.cpp:325-361, then zero
 * the gradient accumulators (:511-517). lr[3] per layer. */
void oracle_update_all(int n1, int n2, int f1, int f2, int f3, float* params,
                       float* grads, float* momentum_bufs, float momentum,
                       float wd, const float* lr, unsigned batch);

/* forward only (inference, ConfigBasedDataPipeline.cpp:114-126 / :200-241),
 * writes A3 [batch][h-pad][w-pad]. */
void oracle_forward(int n1, int n2, int f1, int f2, int f3, const float* X,
                    int w, int h, int batch, const float* params, float* out);

#ifdef __cplusplus
}
#endif
#endif
