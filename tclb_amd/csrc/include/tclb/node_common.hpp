// Small helpers available to every model's dynamics code.
#pragma once
#include "core.hpp"

namespace tclb {

template <class R>
TCLB_FN R sq(R x) { return x * x; }

template <class R>
TCLB_FN vec3<R> make_vec(R x, R y, R z) {
  vec3<R> v;
  v.x = x; v.y = y; v.z = z;
  return v;
}

// Colour map helper used by the GUI/preview path (reference: Color(), e.g.
// models/flow/d3q27/Dynamics.c.Rt:66-76).  Returned as (value, alpha).
template <class R>
struct color2 {
  float x, y;
};

}  // namespace tclb
