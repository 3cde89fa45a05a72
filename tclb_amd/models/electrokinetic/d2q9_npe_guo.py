"""d2q9_npe_guo — electro-kinetic flow: Nernst-Planck ion transport (two species h_0,
h_1), Poisson equation for the electric double-layer potential psi (g) and the external
potential Phi (phi), all as D2Q9 LB schemes (Guo et al.), coupled to a BGK flow f by the
electric body force.  Reference: models/electrokinetic/d2q9_npe_guo/{Dynamics.R,
Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_npe_guo", dims=2, family="electrokinetic", reference="models/electrokinetic/d2q9_npe_guo",
              description="Nernst-Planck-Poisson electro-osmotic flow, five D2Q9 distributions")
    for g in ("phi", "g", "f", "h_0", "h_1"):
        for i, (x, y) in enumerate(U9):
            m.add_density(f"{g}[{i}]", x, y, 0, group=g)
    m.add_quantity("F", vector=True, unit="kgm/s2")
    m.add_quantity("U", vector=True, unit="m/s")
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("n0", unit="An/m3")
    m.add_quantity("n1", unit="An/m3")
    m.add_quantity("Psi", unit="V")
    m.add_quantity("Phi", unit="V")
    m.add_quantity("GradPsi", vector=True, unit="V/m")
    m.add_quantity("GradPhi", vector=True, unit="V/m")
    m.add_quantity("rho_e", unit="C/m3")
    S = m.add_setting
    S("n_inf_0")
    S("n_inf_1")
    S("el", unit="C")
    S("el_kbT", unit="C/J")
    S("epsilon", unit="C2/J/m")
    S("dt")
    S("psi0", unit="V", default=1.0)
    S("phi0", unit="V", default=1.0)
    S("ez", default=1.0)
    S("Ex", unit="V/m", default=0)
    S("D", unit="m2/t", default=1.0 / 6.0, comment="Ion diffusivity")
    S("nu", unit="sPa", comment="viscosity")
    S("rho_bc", unit="kg/m3", default=1, comment="fluid density at  boundary", zonal=True)
    S("phi_bc", unit="V", default=1, comment="phi at  boundary", zonal=True)
    S("psi_bc", unit="V", default=1, comment="psi at  boundary - zeta", zonal=True)
    S("t_to_s", default="1t/s", unit="t/s", comment="time scale ratio")
    m.add_global("TotalMomentum")
    for n in ["SSymmetry", "NSymmetry", "NVelocity", "SVelocity", "WVelocity", "EVelocity"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_density("BC[0]", 0, 0, 0, group="BC")
    m.add_density("BC[1]", 0, 0, 0, group="BC")
    for n in ["EPressure", "Solid", "Wall", "WPressure"]:
        m.add_node_type(n, "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("electrokinetic/d2q9_npe_guo.inc")
    return m
