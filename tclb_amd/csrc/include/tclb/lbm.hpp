// Generic lattice-Boltzmann node operators, templated on a lattice-traits class.
//
// A traits class (emitted per density group by tclb_amd.emit) provides
//   static constexpr int Q, D;  cx(i), cy(i), cz(i), opp(i), w_num(i)/w_den(i) (or w(i))
// Every loop below is over compile-time constants and fully unrolled, so each
// operator compiles to straight-line register code.
//
// Parity notes (reference):
//   bounce_back   ~ FullBounceBack      src/lib/boundary.R:115-145
//   symmetry      ~ Symmetry            src/lib/boundary.R:147-166
//   zouhe         ~ ZouHe               src/lib/boundary.R:180-230 (mode ZH_REF)
//                 ~ ZouHeRewrite        src/lib/boundary.R:262-311 (mode ZH_REWRITE)
//   feq2          ~ MRT_eq(...)$feq at second order (src/lib/feq.R:38-82) for the
//                   standard D2Q9/D3Q19/D3Q27 weights
#pragma once
#include "core.hpp"

namespace tclb {
namespace lbm {

template <class L>
TCLB_FN constexpr int c_(int i, int a) { return a == 0 ? L::cx(i) : (a == 1 ? L::cy(i) : L::cz(i)); }

template <class L, class R>
TCLB_FN R sum(const R* f) {
  R s = R(0);
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) s += f[i];
  return s;
}

template <class L, class R>
TCLB_FN void momentum(const R* f, R& jx, R& jy, R& jz) {
  jx = R(0); jy = R(0); jz = R(0);
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    if (L::cx(i) == 1) jx += f[i];
    if (L::cx(i) == -1) jx -= f[i];
    if (L::cy(i) == 1) jy += f[i];
    if (L::cy(i) == -1) jy -= f[i];
    if (L::cz(i) == 1) jz += f[i];
    if (L::cz(i) == -1) jz -= f[i];
  }
}

// Standard second-order equilibrium in conserved variables (rho, J = rho*u).
template <class L, class R>
TCLB_FN void feq2(R* f, R rho, R jx, R jy, R jz) {
  const R ir = R(1) / rho;
  const R jsq = (jx * jx + jy * jy + jz * jz) * ir;
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    const R cj = R(L::cx(i)) * jx + R(L::cy(i)) * jy + R(L::cz(i)) * jz;
    f[i] = R(L::w(i)) * (rho + R(3) * cj + R(4.5) * cj * cj * ir - R(1.5) * jsq);
  }
}

template <class L, class R>
TCLB_FN void bounce_back(R* f) {
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    const int j = L::opp(i);
    if (i < j) {
      const R t = f[i];
      f[i] = f[j];
      f[j] = t;
    }
  }
}

// mirror index across axis AX
template <class L>
TCLB_FN constexpr int mirror(int i, int ax) {
  for (int j = 0; j < L::Q; j++) {
    bool ok = true;
    for (int a = 0; a < 3; a++) {
      int ci = c_<L>(i, a);
      if (a == ax) ci = -ci;
      if (ci != c_<L>(j, a)) ok = false;
    }
    if (ok) return j;
  }
  return i;
}

// Symmetry(direction = AX+1, sign = SGN): f_i <- f_mirror(i) for SGN*c_i[AX] > 0
template <class L, int AX, int SGN, class R>
TCLB_FN void symmetry(R* f) {
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    if (SGN * c_<L>(i, AX) > 0) f[i] = f[mirror<L>(i, AX)];
  }
}

// ----------------------------------------------------------------------------
// Zou/He type boundary conditions (non-equilibrium bounce-back of the unknowns
// i in sel = {SGN*c_i[AX] > 0}:  f_i = f_opp(i) + 6 w_i c_i.J ).
//   A   = sum_{i !in sel} f_i + sum_{i in sel} f_opp(i)      (= mass of fs at J=0)
//   B_t = sum_{i !in sel} f_i c_it + sum_{i in sel} f_opp(i) c_it
//   K   = 6 sum_{sel} w c_AX     T_t = 6 sum_{sel} w c_t^2
// ZH_REF     : J_t solves sum fs c_t = J_t             -> J_t = B_t / (1 - T_t)
// ZH_REWRITE : sum fs c_t = 0 (no tangential velocity) -> J_t = -B_t / T_t
// velocity   : J_AX = rho V, sum fs = rho              -> rho = A / (1 - K V)
// pressure   : rho = rho0                             -> J_AX = (rho0 - A) / K
// ----------------------------------------------------------------------------
enum { ZH_REF = 0, ZH_REWRITE = 1 };

template <class L>
TCLB_FN constexpr double zh_K(int ax, int sgn) {
  double s = 0;
  for (int i = 0; i < L::Q; i++)
    if (sgn * c_<L>(i, ax) > 0) s += 6.0 * L::w(i) * c_<L>(i, ax);
  return s;
}
template <class L>
TCLB_FN constexpr double zh_T(int ax, int sgn, int t) {
  double s = 0;
  for (int i = 0; i < L::Q; i++)
    if (sgn * c_<L>(i, ax) > 0) s += 6.0 * L::w(i) * c_<L>(i, t) * c_<L>(i, t);
  return s;
}

template <class L, int AX, int SGN, int MODE, class R>
TCLB_FN void zouhe(R* f, bool pressure, R value, R& rho_out, R* J, const R* vt = nullptr) {
  R A = R(0);
  R B[3] = {R(0), R(0), R(0)};
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    const bool sel = SGN * c_<L>(i, AX) > 0;
    const R v = sel ? f[L::opp(i)] : f[i];
    A += v;
    TCLB_UNROLL for (int t = 0; t < L::D; t++) {
      if (t == AX) continue;
      if (c_<L>(i, t) != 0) B[t] += R(c_<L>(i, t)) * v;
    }
  }
  constexpr double K = zh_K<L>(AX, SGN);
  R rho;
  if (pressure) {
    rho = value;
    J[AX] = (rho - A) * R(1.0 / K);
  } else {
    rho = A / (R(1) - R(K) * value);
    J[AX] = rho * value;
  }
  TCLB_UNROLL for (int t = 0; t < L::D; t++) {
    if (t == AX) continue;
    const double T = zh_T<L>(AX, SGN, t);
    if (MODE == ZH_REF) {
      J[t] = B[t] * R(1.0 / (1.0 - T));
      if (vt != nullptr) J[t] += rho * vt[t];
    } else {
      // ZouHeRewrite: sum fs c_t = rho vt_t  ->  J_t = (rho vt_t - B_t) / T_t
      J[t] = ((vt != nullptr ? rho * vt[t] : R(0)) - B[t]) * R(1.0 / T);
    }
  }
  if (L::D < 3) J[2] = R(0);
  if (L::D < 2) J[1] = R(0);
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    if (SGN * c_<L>(i, AX) > 0) {
      R cj = R(0);
      TCLB_UNROLL for (int a = 0; a < L::D; a++)
        if (c_<L>(i, a) != 0) cj += R(c_<L>(i, a)) * J[a];
      f[i] = f[L::opp(i)] + R(6.0 * L::w(i)) * cj;
    }
  }
  rho_out = rho;
}

// Non-equilibrium bounce-back with the tangential momentum taken from the in-plane
// populations as J_t = -3 sum_{c_AX = 0} c_t f  (the hand-written D3Q27 Zou/He blocks
// of reference models/flow/experimental/d3q27_BGK/Dynamics.c:174-351,
// models/nonnewtonian/d3q27_viscoplastic/Dynamics.c:175-325 and
// models/nonnewtonian/d3q27_kl/Dynamics.c.Rt:144-259 use exactly this closure).
// rho/J_AX closure as in zouhe(): velocity -> rho = A/(1-K V), pressure -> J_AX = (rho-A)/K.
template <class L, int AX, int SGN, class R>
TCLB_FN void nebb_plane(R* f, bool pressure, R value, R* Jout = nullptr, R* rho_out = nullptr) {
  R A = R(0);
  R Jt[3] = {R(0), R(0), R(0)};
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    const bool sel = SGN * c_<L>(i, AX) > 0;
    A += sel ? f[L::opp(i)] : f[i];
    if (c_<L>(i, AX) == 0) {
      TCLB_UNROLL for (int t = 0; t < 3; t++)
        if (t != AX && c_<L>(i, t) != 0) Jt[t] += R(c_<L>(i, t)) * f[i];
    }
  }
  constexpr double K = zh_K<L>(AX, SGN);
  R J[3];
  TCLB_UNROLL for (int t = 0; t < 3; t++) J[t] = R(-3) * Jt[t];
  R rho = value;
  if (pressure) {
    J[AX] = (value - A) * R(1.0 / K);
  } else {
    rho = A / (R(1) - R(K) * value);
    J[AX] = rho * value;
  }
  if (Jout != nullptr) { Jout[0] = J[0]; Jout[1] = J[1]; Jout[2] = J[2]; }
  if (rho_out != nullptr) *rho_out = rho;
  TCLB_UNROLL for (int i = 0; i < L::Q; i++) {
    if (SGN * c_<L>(i, AX) > 0) {
      R cj = R(0);
      TCLB_UNROLL for (int a = 0; a < 3; a++)
        if (c_<L>(i, a) != 0) cj += R(c_<L>(i, a)) * J[a];
      f[i] = f[L::opp(i)] + R(6.0 * L::w(i)) * cj;
    }
  }
}

}  // namespace lbm
}  // namespace tclb
