// Automatic differentiation of node updates (adjoint / tangent support).
//
// The reference generates adjoint node code with Tapenade per model (tools/makeAD,
// ADJOINT=1 models only).  Here every model is differentiable: the node code is
// templated on the real type R, and instantiating it with Dual<double, K> (K forward
// tangents) yields the local Jacobian of one node update with respect to every value the
// node loaded (populations, stencil fields, seeded settings).  The adjoint executor then
// scatters  a_in(load site) += a_out(store) * d store / d load  — the transpose of the
// stencil update — plus d Objective / d load, and accumulates setting gradients.
// Non-AD builds use AdRec<R> below, whose hooks compile to nothing.
#pragma once
#include <cmath>
#include "core.hpp"

namespace tclb {

template <class T, int K>
struct Dual {
  T v;
  T d[K];
  TCLB_FN Dual() : v(0) { for (int k = 0; k < K; k++) d[k] = T(0); }
  TCLB_FN Dual(T x) : v(x) { for (int k = 0; k < K; k++) d[k] = T(0); }
  template <class U>
  TCLB_FN explicit operator U() const { return U(v); }

  TCLB_FN Dual& operator+=(const Dual& b) { v += b.v; for (int k = 0; k < K; k++) d[k] += b.d[k]; return *this; }
  TCLB_FN Dual& operator-=(const Dual& b) { v -= b.v; for (int k = 0; k < K; k++) d[k] -= b.d[k]; return *this; }
  TCLB_FN Dual& operator*=(const Dual& b) {
    for (int k = 0; k < K; k++) d[k] = d[k] * b.v + v * b.d[k];
    v *= b.v;
    return *this;
  }
  TCLB_FN Dual& operator/=(const Dual& b) {
    const T iv = T(1) / b.v, q = v * iv;
    for (int k = 0; k < K; k++) d[k] = (d[k] - q * b.d[k]) * iv;
    v = q;
    return *this;
  }
  friend TCLB_FN Dual operator+(Dual a, const Dual& b) { return a += b; }
  friend TCLB_FN Dual operator-(Dual a, const Dual& b) { return a -= b; }
  friend TCLB_FN Dual operator*(Dual a, const Dual& b) { return a *= b; }
  friend TCLB_FN Dual operator/(Dual a, const Dual& b) { return a /= b; }
  friend TCLB_FN Dual operator-(const Dual& a) {
    Dual r;
    r.v = -a.v;
    for (int k = 0; k < K; k++) r.d[k] = -a.d[k];
    return r;
  }
  friend TCLB_FN Dual operator+(const Dual& a) { return a; }
  friend TCLB_FN bool operator<(const Dual& a, const Dual& b) { return a.v < b.v; }
  friend TCLB_FN bool operator>(const Dual& a, const Dual& b) { return a.v > b.v; }
  friend TCLB_FN bool operator<=(const Dual& a, const Dual& b) { return a.v <= b.v; }
  friend TCLB_FN bool operator>=(const Dual& a, const Dual& b) { return a.v >= b.v; }
  friend TCLB_FN bool operator==(const Dual& a, const Dual& b) { return a.v == b.v; }
  friend TCLB_FN bool operator!=(const Dual& a, const Dual& b) { return a.v != b.v; }
  friend TCLB_FN bool operator!(const Dual& a) { return !a.v; }

  // chain rule helper: f(v), f'(v)
  TCLB_FN Dual chain(T fv, T dfv) const {
    Dual r;
    r.v = fv;
    for (int k = 0; k < K; k++) r.d[k] = dfv * d[k];
    return r;
  }
  friend TCLB_FN Dual sqrt(const Dual& a) { const T s = std::sqrt(a.v); return a.chain(s, s > T(0) ? T(0.5) / s : T(0)); }
  friend TCLB_FN Dual exp(const Dual& a) { const T e = std::exp(a.v); return a.chain(e, e); }
  friend TCLB_FN Dual log(const Dual& a) { return a.chain(std::log(a.v), T(1) / a.v); }
  friend TCLB_FN Dual sin(const Dual& a) { return a.chain(std::sin(a.v), std::cos(a.v)); }
  friend TCLB_FN Dual cos(const Dual& a) { return a.chain(std::cos(a.v), -std::sin(a.v)); }
  friend TCLB_FN Dual tan(const Dual& a) { const T t = std::tan(a.v); return a.chain(t, T(1) + t * t); }
  friend TCLB_FN Dual tanh(const Dual& a) { const T t = std::tanh(a.v); return a.chain(t, T(1) - t * t); }
  friend TCLB_FN Dual sinh(const Dual& a) { return a.chain(std::sinh(a.v), std::cosh(a.v)); }
  friend TCLB_FN Dual cosh(const Dual& a) { return a.chain(std::cosh(a.v), std::sinh(a.v)); }
  friend TCLB_FN Dual asin(const Dual& a) { return a.chain(std::asin(a.v), T(1) / std::sqrt(T(1) - a.v * a.v)); }
  friend TCLB_FN Dual acos(const Dual& a) { return a.chain(std::acos(a.v), T(-1) / std::sqrt(T(1) - a.v * a.v)); }
  friend TCLB_FN Dual log1p(const Dual& a) { return a.chain(std::log1p(a.v), T(1) / (T(1) + a.v)); }
  friend TCLB_FN Dual expm1(const Dual& a) { return a.chain(std::expm1(a.v), std::exp(a.v)); }
  friend TCLB_FN Dual atan(const Dual& a) { return a.chain(std::atan(a.v), T(1) / (T(1) + a.v * a.v)); }
  friend TCLB_FN Dual fabs(const Dual& a) { return a.chain(std::fabs(a.v), a.v < T(0) ? T(-1) : T(1)); }
  friend TCLB_FN Dual abs(const Dual& a) { return fabs(a); }
  friend TCLB_FN Dual cbrt(const Dual& a) { const T c = std::cbrt(a.v); return a.chain(c, c != T(0) ? c / (T(3) * a.v) : T(0)); }
  friend TCLB_FN Dual floor(const Dual& a) { return Dual(std::floor(a.v)); }
  friend TCLB_FN Dual pow(const Dual& a, const Dual& b) {
    const T p = std::pow(a.v, b.v);
    Dual r;
    r.v = p;
    const T da = a.v != T(0) ? b.v * std::pow(a.v, b.v - T(1)) : T(0);
    const T db = a.v > T(0) ? p * std::log(a.v) : T(0);
    for (int k = 0; k < K; k++) r.d[k] = da * a.d[k] + db * b.d[k];
    return r;
  }
  friend TCLB_FN Dual atan2(const Dual& y, const Dual& x) {
    const T r2 = x.v * x.v + y.v * y.v;
    Dual r;
    r.v = std::atan2(y.v, x.v);
    for (int k = 0; k < K; k++) r.d[k] = r2 > T(0) ? (x.v * y.d[k] - y.v * x.d[k]) / r2 : T(0);
    return r;
  }
  friend TCLB_FN Dual fmax(const Dual& a, const Dual& b) { return a.v >= b.v ? a : b; }
  friend TCLB_FN Dual fmin(const Dual& a, const Dual& b) { return a.v <= b.v ? a : b; }
};

template <class R>
struct is_dual { static constexpr bool value = false; };
template <class T, int K>
struct is_dual<Dual<T, K>> { static constexpr bool value = true; };

// Adjoint context (Launch::ext[5] in AD launches)
struct AdCtx {
  const double* aout;      // adjoint of the stage outputs  [nfields][field]
  double* ain;             // adjoint of the stage inputs   [nfields][field] (accumulated)
  double* gset;            // d J / d global setting        [NSETTINGS]
  double* gzon;            // d J / d zonal setting         [NZSETTINGS][nzones]
  const int* set_mask;     // seed these global settings    [NSETTINGS] (nullable)
  const int* zon_mask;     // seed these zonal settings     [NZSETTINGS] (nullable)
  double obj_weight;       // adjoint seed of the Objective global
  int overflow;            // set when a node needed more than K tangents
  int reserved;
};

// Adjoint push of a hand-written reverse sweep (Model.set_reverse): a += v at an input's
// load site (device fp64 atomic / OpenMP atomic).
TCLB_FN void ad_push(double* p, double v) {
  if (v == 0.0) return;
#if TCLB_GPU && defined(__HIP_DEVICE_COMPILE__)
  unsafeAtomicAdd(p, v);
#else
#pragma omp atomic
  *p += v;
#endif
}
// a node type with a reverse sweep (the emitter defines HAS_REV for models that have one)
template <class N, class = void>
struct has_rev { static constexpr bool value = false; };
template <class N>
struct has_rev<N, decltype((void)N::HAS_REV)> { static constexpr bool value = N::HAS_REV; };

// Recorder of seeded inputs; no-op for plain real types.
template <class R>
struct AdRec {
  TCLB_FN void init(const Launch&) {}
  TCLB_FN R load(double v, int, long long) { return R(v); }
  TCLB_FN R setting(int, R v) { return v; }
  TCLB_FN R zonal(int, int, R v) { return v; }
  TCLB_FN void store(int, long long, const R&) {}
};

#if !TCLB_GPU
template <class T, int K>
struct AdRec<Dual<T, K>> {
  typedef Dual<T, K> D;
  AdCtx* ctx = nullptr;
  long long fs = 0;
  long long zonal_pitch = 0;
  int n = 0;
  int kind[K];      // 0 load, 1 global setting, 2 zonal setting
  int fi[K];
  long long idx[K];
  void init(const Launch& L) {
    ctx = (AdCtx*)L.ext[5];
    fs = L.fs;
    zonal_pitch = L.nzones;
    n = 0;
  }
  D seed(double v, int k_kind, int f, long long i) {
    D r(v);
    if (n < K) {
      r.d[n] = T(1);
      kind[n] = k_kind; fi[n] = f; idx[n] = i;
      n++;
    } else if (ctx) {
      ctx->overflow = 1;
    }
    return r;
  }
  D load(double v, int f, long long i) {
    if (!ctx) return D(v);
    for (int k = 0; k < n; k++)   // the same site read twice shares its tangent
      if (kind[k] == 0 && fi[k] == f && idx[k] == i) { D r(v); r.d[k] = T(1); return r; }
    return seed(v, 0, f, i);
  }
  D setting(int i, D v) {
    if (ctx && ctx->set_mask && ctx->set_mask[i]) return seed(v.v, 1, i, 0);
    return v;
  }
  D zonal(int i, int zone, D v) {
    if (ctx && ctx->zon_mask && ctx->zon_mask[i]) {
      for (int k = 0; k < n; k++)   // one tangent per (setting, zone) and node
        if (kind[k] == 2 && fi[k] == i && idx[k] == zone) { D r(v.v); r.d[k] = T(1); return r; }
      return seed(v.v, 2, i, zone);
    }
    return v;
  }
  // route a * d(value)/d(input k) to the adjoint of input k
  void scatter(double a, const D& val) {
    if (a == 0.0) return;
    for (int k = 0; k < n; k++) {
      const double c = a * (double)val.d[k];
      if (c == 0.0) continue;
      double* dst = kind[k] == 0 ? ctx->ain + (long long)fi[k] * fs + idx[k]
                  : (kind[k] == 1 ? ctx->gset + fi[k] : ctx->gzon + (long long)fi[k] * zonal_pitch + idx[k]);
#pragma omp atomic
      *dst += c;
    }
  }
  void store(int f, long long node, const D& val) {
    if (!ctx) return;
    scatter(ctx->aout[(long long)f * fs + node], val);
  }
};
#endif

}  // namespace tclb
