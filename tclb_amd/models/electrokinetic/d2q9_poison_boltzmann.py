"""d2q9_poison_boltzmann — Poisson-Boltzmann equation for the electric double-layer
potential psi solved as a D2Q9 lattice-Boltzmann scheme (Wang-Kang), with the Boltzmann
charge density rho_e = -2 n_inf z e sinh(z e psi / kT) as source.  Three-stage Iteration
(BaseIteration, CalcPsi, CalcSubiter).
Reference: models/electrokinetic/d2q9_poison_boltzmann/{Dynamics.R, Dynamics.c.Rt}."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_poison_boltzmann", dims=2, family="electrokinetic",
              reference="models/electrokinetic/d2q9_poison_boltzmann",
              description="Poisson-Boltzmann double-layer potential as a D2Q9 LB scheme")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"g[{i}]", x, y, 0, group="g")
    m.add_density("subiter", 0, 0, 0, group="subiter")
    m.add_field("psi", stencil2d=1)
    m.add_quantity("Psi")
    m.add_quantity("Subiter")
    m.add_stage("BaseIteration", "Run", save_fields=["g"], load_densities=["g"])
    m.add_stage("CalcPsi", "CalcPsi", save_fields=["psi"], load_densities=["g"])
    m.add_stage("CalcSubiter", "CalcSubiter", save_fields=["subiter"], load_densities=["subiter"])
    m.add_action("Iteration", ["BaseIteration", "CalcPsi", "CalcSubiter"])
    m.add_quantity("rho_e", unit="kg/m3")
    S = m.add_setting
    S("tau_psi", comment="tau_psi")
    for n in ["n_inf", "z", "el", "kb", "T", "epsilon", "dt"]:
        S(n)
    S("psi_bc", default=1, comment="psi at  boundary - zeta", zonal=True)
    S("psi0", default=1, comment="initial psi - zeta", zonal=True)
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("Collision", "COLLISION")
    m.set_dynamics("electrokinetic/d2q9_poison_boltzmann.inc")
    return m
