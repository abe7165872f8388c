// Shared by the fp32 (mlp.hip) and bf16 (mlp_bf16.hip) MLP paths: the packed fp32 parameter layout both
// consume (one flat buffer per network: coarse | fine in the trainer), split-M sizing, head activations.
#pragma once
#include "common.hpp"

namespace nerf_mlp {

constexpr int NT = 22;  // tensors in the packed layout
constexpr int KPAD[8] = {64, 256, 256, 256, 320, 256, 256, 256};
constexpr int KREAL[8] = {63, 256, 256, 256, 319, 256, 256, 256};

struct Layout {
  int64_t off[NT];
  int rows[NT], cols[NT], creal[NT];
  int64_t total;
};

inline Layout make_layout() {
  Layout L{};
  int64_t o = 0;
  int t = 0;
  auto add = [&](int r, int c, int cr) {
    L.off[t] = o; L.rows[t] = r; L.cols[t] = c; L.creal[t] = cr;
    o += (int64_t)r * c;
    o = (o + 31) & ~int64_t(31);  // keep every tensor 128-B aligned
    ++t;
  };
  for (int i = 0; i < 8; ++i) {
    add(256, KPAD[i], KREAL[i]);
    add(256, 1, 1);
  }
  add(32, 256, 256);  // head W: row 0 sigma_head, rows 1..15 geo_head
  add(32, 1, 1);
  add(128, 64, 42);   // color_mlp.layer0
  add(128, 1, 1);
  add(32, 128, 128);  // color_mlp.color_out (rows 0..2)
  add(32, 1, 1);
  L.total = o;
  return L;
}

inline const Layout& layout() {
  static const Layout L = make_layout();
  return L;
}

inline int64_t round_up(int64_t a, int64_t b) { return (a + b - 1) / b * b; }

// split-M partial slabs of the weight gradient: one per NERF_SPLIT_ROWS rows, at most 256
#ifndef NERF_SPLIT_ROWS  // 1024: the split weight-gradient GEMM runs one workgroup per split, so the coarse net
#define NERF_SPLIT_ROWS 1024  // (Mp = 262,144) needs 256 splits to fill the CUs
#endif
inline int n_splits(int64_t Mp) {
  int64_t s = Mp / NERF_SPLIT_ROWS;
  if (s < 1) s = 1;
  if (s > 256) s = 256;
  return (int)s;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }
constexpr float EXP_MAX = 88.722839111f;  // trunc_exp clamp for fp32 (models/trunc_exp.py:30-61)

}  // namespace nerf_mlp

#define TRY(x)                     \
  do {                             \
    int _e = (x);                  \
    if (_e != NERF_OK) return _e;  \
  } while (0)
