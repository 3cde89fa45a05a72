"""d2q9_reaction_diffusion_system — a family of diffusion-reaction systems on D2Q9:
diffusing species (DREs, one D2Q9 population set each) coupled to local ODE species
(stored fields), with the reaction source integrated by Trapezoid (implicit phi
reconstruction), Euler, Heun or Midpoint rules and SRT or TRT ("TRT_M", magic parameter)
collisions.  Systems (reference option names): AllenCahn, SIR_SimpleLaplace,
SIR_ModifiedPeng (diffusing W + ODEs S, I, R, N), SimpleDiffusion, LinearReaction.
Reference: models/reaction/d2q9_reaction_diffusion_system/{Dynamics.R, Dynamics.c.Rt}
(OPT="(AllenCahn+SIR_ModifiedPeng+SIR_SimpleLaplace+SimpleDiffusion+LinearReaction)*
(Trapezoidal+Midpoint+Heun+Euler)-1").

Deviation (documented): the SIR_ModifiedPeng Newton step solves the full 3x3 Jacobian
(the reference calls Eigen's ldlt() on a non-symmetric Jacobian, which reads only its
lower triangle); both iterate to the same implicit-trapezoid root within the 1e-5
residual tolerance.
"""
from ..dsl import Model

SYSTEMS = {
    "AllenCahn": (["PHI"], [], ["Lambda"]),
    "SIR_SimpleLaplace": (["S", "I", "R"], [], ["Beta", "Gamma"]),
    "SIR_ModifiedPeng": (["W"], ["S", "I", "R", "N"], ["Beta", "Beta_w", "Gamma"]),
    "SimpleDiffusion": (["PHI"], [], []),
    "LinearReaction": (["PHI"], [], ["LinearReactionRate"]),
}
INTEGRATORS = {"Trapezoid": 0, "Euler": 1, "Heun": 2, "Midpoint": 3}
CV = (0, 1, -1)


def build(system: str = "AllenCahn", integrator: str = "Trapezoid") -> Model:
    dres, odes, params = SYSTEMS[system]
    m = Model(f"d2q9_reaction_diffusion_system_{system}", dims=2, family="reaction",
              reference="models/reaction/d2q9_reaction_diffusion_system",
              description=f"D2Q9 diffusion-reaction system {system} ({integrator} source integration)")
    for i in range(len(dres)):
        for k in range(9):
            px, py = k % 3, k // 3
            m.add_density(f"dre_{i + 1}[{k}]", CV[px], CV[py], 0, group=f"dre_{i + 1}",
                          comment=f"LB density dre_{i + 1}_f{px}{py}0")
    for i, name in enumerate(odes):
        m.add_field(f"ode_{i + 1}", dx=(-1, 1), dy=(-1, 1))
        m.add_density(f"Init_{name}_External", 0, 0, 0, group="init", parameter=True)
    for name in dres:
        m.add_quantity(name, unit="1")
        m.add_density(f"Init_{name}_External", 0, 0, 0, group="init", parameter=True)
    for name in odes:
        m.add_quantity(name, unit="1")
        m.add_setting(f"Init_{name}", zonal=True)
    m.add_stage("InitFromExternal", "InitFromExternal", load_densities=True, save_fields=True)
    m.add_action("InitFromExternalAction", ["InitFromExternal"])
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("SRT_DF", "COLLISION")
    m.add_node_type("TRT_M", "COLLISION")
    m.add_setting("magic_parameter", default=1.0 / 6.0,
                  comment="to control relaxation frequency of even moments in TRT collision kernel")
    for name in dres:
        m.add_setting(f"Init_{name}", zonal=True)
        m.add_setting(f"Diffusivity_{name}", default=0.02, comment=f"Diffusivity for {name}")
    for p in params:
        m.add_setting(p, default=0.0, comment=f"Model parameter {p}")
    m.defines = {"RD_NDRE": str(len(dres)), "RD_NODE": str(len(odes)),
                 "RD_SYSTEM_" + system: "1", "RD_INTEGRATOR": str(INTEGRATORS[integrator])}
    m.options = {system: True, integrator: True}
    m.set_dynamics("reaction/d2q9_reaction_diffusion_system.inc")
    return m
