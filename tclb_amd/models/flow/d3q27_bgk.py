"""d3q27_BGK / d3q27_BGK_galcor — experimental D3Q27 single-relaxation models with a
Kupershtokh (exact-difference) body force and slice-integral globals.

* ``d3q27_BGK``: second-order polynomial equilibrium
  (reference models/flow/experimental/d3q27_BGK/{Dynamics.R, Dynamics.c}).
* ``d3q27_BGK_galcor``: product-form equilibrium with the Galilean correction of the
  diagonal second moments (reference models/flow/experimental/d3q27_BGK_galcor).

Storage order is the reference's expand.grid order: k = px + 3 py + 9 pz with
p = 0,1,2 <-> c = 0,+1,-1 (field f[k] is the reference's f<px><py><pz>).
"""
import numpy as np

from ..dsl import Model

CV = (0, 1, -1)
P = np.array([[k % 3, (k // 3) % 3, k // 9] for k in range(27)])
U = np.array([[CV[a], CV[b], CV[c]] for a, b, c in P])


def add_slice_globals(m: Model):
    for pl in ("XY", "XZ", "YZ"):
        for q, u in (("vx", "m3/s"), ("vy", "m3/s"), ("vz", "m3/s"), ("rho1", "kg/m"), ("rho2", "kg/m"),
                     ("area", "m2")):
            m.add_global(f"{pl}{q}", comment="Volume flux", unit=u)


def build(galcor: bool = False) -> Model:
    name = "d3q27_BGK_galcor" if galcor else "d3q27_BGK"
    m = Model(name, dims=3, family="flow", reference=f"models/flow/experimental/{name}",
              description="D3Q27 BGK" + (" with Galilean-corrected product equilibrium" if galcor else "")
              + ", Kupershtokh forcing")
    for k in range(27):
        m.add_density(f"f[{k}]", int(U[k, 0]), int(U[k, 1]), int(U[k, 2]), group="f",
                      comment=f"density F{P[k, 0]}{P[k, 1]}{P[k, 2]}")
    m.add_quantity("P", unit="Pa")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_setting("nu", default=0.16666666, comment="Viscosity")
    m.add_setting("Velocity", default="0m/s", comment="Inlet velocity", zonal=True, unit="m/s")
    m.add_setting("Pressure", default="0Pa", comment="Inlet pressure", zonal=True, unit="Pa")
    m.add_setting("GalileanCorrection", default=0.0, comment="Galilean correction term")
    for a in "XYZ":
        m.add_setting(f"Force{a}", default=0, comment=f"Force {a}")
    for n in ("XYslice1", "XZslice1", "YZslice1", "XYslice2", "XZslice2", "YZslice2"):
        m.add_node_type(n, "ADDITIONALS")
    m.add_global("Flux", comment="Volume flux", unit="m3/s")
    m.add_global("TotalRho", comment="Total mass", unit="kg")
    add_slice_globals(m)
    for n in ("SymmetryY", "SymmetryZ", "TopSymmetry", "BottomSymmetry", "NVelocity", "SVelocity", "NPressure",
              "SPressure", "EPressure", "EVelocity", "Solid", "Wall", "WPressure", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.options = {"GALCOR": galcor}
    m.set_dynamics("flow/d3q27_bgk.inc")
    return m
