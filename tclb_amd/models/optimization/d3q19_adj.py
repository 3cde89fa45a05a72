"""d3q19_adj — D3Q19 d'Humieres MRT (incompressible equilibria, rho0 = 1) with a porosity
design field w that damps the momentum by w^Theta — the 3-D topology-optimisation model;
flux/energy/pressure objectives on Inlet/Outlet nodes, material penalty on DesignSpace.
Gradients come from the generic AD adjoint.
Reference: models/optimization/d3q19_adj/{Dynamics.R, Dynamics.c.Rt} (ADJOINT=1)."""
from ..dsl import Model
from ...emit.symbolic import d3q19_mrt
from ..flow.d3q19 import mrt19_block
from ...emit.blocks import dense_transform


def mrt19_transposes(_m):
    """transposes of the moment maps for the reverse sweep (rev_run): a_f = M^T a_m and
    a_m = (M^-1)^T a_f"""
    M = d3q19_mrt().MAT
    return "\n".join([dense_transform("mrt_moments_T", M.T, 19, 19, "a_f = a_m . MRTMAT^T"),
                      dense_transform("mrt_inverse_T", M.inv().T, 19, 19, "a_m = a_f . (MRTMAT^-1)^T")])


def build() -> Model:
    m = Model("d3q19_adj", dims=3, family="optimization", reference="models/optimization/d3q19_adj",
              description="D3Q19 incompressible MRT with a porosity design field (3-D topology optimisation)")
    U = d3q19_mrt().U
    for i in range(19):
        m.add_density(f"f[{i}]", int(U[i, 0]), int(U[i, 1]), int(U[i, 2]), group="f", comment=f"density F{i}")
    m.add_density("w", 0, 0, 0, group="w", parameter=True, comment="weight fluid-solid")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("W")
    m.add_quantity("WB", adjoint=True)
    S = m.add_setting
    S("omega", comment="one over relaxation time")
    S("nu", default=0.16666666, comment="viscosity", omega="1.0/(3*nu + 0.5)")
    S("InletVelocity", default="0m/s", comment="inlet velocity", unit="m/s")
    S("InletPressure", default="0Pa", comment="inlet pressure", unit="Pa", InletDensity="1.0+InletPressure/3")
    S("InletDensity", default=1, comment="inlet density")
    S("Theta", default=1, comment="porosity exponent")
    for g in ("Flux", "EnergyFlux", "PressureFlux", "PressureDiff"):
        m.add_global(g, comment="pressure loss")
    m.add_global("MaterialPenalty", comment="quadratic penalty for intermediate material parameter")
    m.add_node_type("Inlet", "OBJECTIVE")
    m.add_node_type("Outlet", "OBJECTIVE")
    for n in ("EPressure", "Solid", "Wall", "WPressure", "WPressureL", "WVelocity"):
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("BGK", "COLLISION")
    m.add_node_type("MRT", "COLLISION")
    m.add_node_type("DesignSpace", "DESIGNSPACE")
    m.add_codegen(mrt19_block)
    m.add_codegen(mrt19_transposes)
    m.set_dynamics("optimization/d3q19_adj.inc")
    m.set_reverse("Run", "rev_ok_run", "rev_run")
    return m
