// runs.hpp -- the pixel order of the split-bf16 fused step (l12x6.hpp,
// d1x6.hpp), included by train_fused.hip inside namespace srcnn::fused.
//
// The 32 slots of a chunk are 8 RUNS of 4 output pixels, and every run lies
// along one image row or one image column, so the 4 X values of a run under
// any tap are consecutive in a pair image (d1x6's gW1 operand: one
// ds_read2_b32 per run and part).  Rows come first, cut into ow / 4 runs
// each; the ow % 4 remainder columns follow, cut into ceil(oh / 4) runs each
// (slots past the tile are dummies: no output, zero delta).  For 33x33 tiles
// (ow = oh = 25): 150 row runs + 7 column runs = 157 runs, 20 chunks, the
// same count as 32 flat pixels per chunk.
struct RunGeom {
  int ow, oh, a, b, cr, nrow, nrun, nch;
  float inv_a, inv_cr;  // reciprocals for the slot -> pixel divisions
};

inline RunGeom run_geom(int ow, int oh) {
  RunGeom r;
  r.ow = ow;
  r.oh = oh;
  r.a = ow / 4;
  r.b = ow % 4;
  r.cr = (oh + 3) / 4;
  r.nrow = r.a * oh;
  r.nrun = r.nrow + r.b * r.cr;
  r.nch = (r.nrun + 7) / 8;
  r.inv_a = r.a ? 1.0f / r.a : 0.0f;
  r.inv_cr = 1.0f / r.cr;
  return r;
}

// k / d for 0 <= k < 2^20 and small d through the float reciprocal (the
// half-integer offset keeps the product off integer boundaries)
__device__ __forceinline__ int run_div(int k, float inv) { return (int)(((float)k + 0.5f) * inv); }

// run k (< nrun) -> first pixel and orientation
__device__ __forceinline__ void run_origin(const RunGeom& r, int k, int& iy, int& ix, bool& col) {
  if (k < r.nrow) {
    iy = run_div(k, r.inv_a);
    ix = 4 * (k - iy * r.a);
    col = false;
  } else {
    k -= r.nrow;
    const int cb = run_div(k, r.inv_cr);
    iy = 4 * (k - cb * r.cr);
    ix = 4 * r.a + cb;
    col = true;
  }
}

// slot s of chunk c -> its pixel (iy, ix); false for a dummy slot (then
// pixel (0, 0), a valid address)
__device__ __forceinline__ bool slot_coord(const RunGeom& r, int c, int s, int& iy, int& ix) {
  const int k = 8 * c + (s >> 2), i = s & 3;
  bool col;
  run_origin(r, k < r.nrun ? k : 0, iy, ix, col);
  if (col)
    iy += i;
  else
    ix += i;
  const bool ok = k < r.nrun && iy < r.oh;
  if (!ok) iy = ix = 0;
  return ok;
}

// slot s of chunk c -> output pixel iy * ow + ix, or -1 for a dummy slot
__device__ __forceinline__ int slot_pixel(const RunGeom& r, int c, int s) {
  const int k = 8 * c + (s >> 2), i = s & 3;
  if (k >= r.nrun) return -1;
  int iy, ix;
  bool col;
  run_origin(r, k, iy, ix, col);
  if (col)
    iy += i;
  else
    ix += i;
  return iy < r.oh ? iy * r.ow + ix : -1;
}
