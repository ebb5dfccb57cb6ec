// The Adam element update and the weight-image refresh shared by the Adam kernels (csrc/optim.hip)
// and the fused slab reduction in the wgrad launch's tail (csrc/wgrad.hip): one definition, so
// every path rounds identically (chief.py:17-20: Adam on the summed gradient).
#pragma once
#include "kernels.h"
#include "common.h"

namespace {

// One Adam element update, shared by both Adam kernels so that they round identically (explicit
// fmaf: no contraction choice is left to the compiler).  Returns the new parameter.
DEV float adam_elem(float& m, float& v, float p, float gi, float b1, float b2, float step_size, float rbc2,
                    float eps) {
  const float mi = fmaf(b1, m, (1.f - b1) * gi);
  const float vi = fmaf(b2, v, (1.f - b2) * (gi * gi));
  m = mi;
  v = vi;
  return p - step_size * mi / fmaf(sqrtf(vi), rbc2, eps);
}

// fp8 mode: the e4m3 image the update's fc1 reads, refreshed with every Adam step (scale: the
// iteration's per-layer qscale, as pack_fp8_kernel; e4m3 conversion saturates)
DEV void f8_put(const F8Shadow& f8, int i, int wi, int wti, float pi) {
  if (f8.img != nullptr) {
    const uint8_t q = Prec<DT_FP8>::cvt(__fdiv_rn(pi, f8.qs[f8.lid[i]]));
    f8.img[wi] = q;
    if (wti >= 0) f8.img[wti] = q;
  }
}


// The Adam step of element i from its gradient gi (its optimizer state already loaded): the
// gradient, m, v, the parameter and its weight-image entries (wti -1: no transposed image, the
// first layer of a head).  The gather + Adam kernel and the wgrad launch's fused tail both use it.
template <int DT>
DEV void adam_apply(int i, float gi, float mi, float vi, float pv, int wi, int wti, float* g, float* p, float* m,
                    float* v, float b1, float b2, float step_size, float rbc2, float eps,
                    typename Prec<DT>::T* wimg, const float* qmul, const F8Shadow& f8) {
  g[i] = gi;
  const float pi = adam_elem(mi, vi, pv, gi, b1, b2, step_size, rbc2, eps);
  m[i] = mi;
  v[i] = vi;
  p[i] = pi;
  if (wi >= 0) {
    const float q = qmul ? pi * qmul[i] : pi;
    Prec<DT>::put(wimg, wi, q);
    if (wti >= 0) Prec<DT>::put(wimg, wti, q);
    f8_put(f8, i, wi, wti, pi);
  }
}

}  // namespace
