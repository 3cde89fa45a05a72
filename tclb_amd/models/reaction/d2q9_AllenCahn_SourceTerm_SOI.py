"""d2q9_AllenCahn_SourceTerm_SOI — advection-diffusion-reaction of a phase field with the
Allen-Cahn source Q = lambda phi (1 - phi^2) (or linear decay Q = -lambda phi with option
``ExpotentialDecay``) integrated to second order (implicit phi reconstruction, "SOI"),
with four collision kernels: SRT_DF_SOI / SRT_M_SOI (BGK in populations / raw moments),
TRT_M_SOI (raw moments, magic-parameter even rate) and TRT_CM_SOI (central moments).
Reference: models/reaction/d2q9_AllenCahn_SourceTerm_SOI/{Dynamics.R, Dynamics.c.Rt}.

Kept as in the reference: boundary routines (Wall, DirichletEQ) exist but Run does not
call them (Dynamics.c.Rt:151), and the Gaussian-hill settings are declared but unused.
"""
from ..dsl import Model

CV = (0, 1, -1)


def build(expdecay: bool = False) -> Model:
    m = Model("d2q9_AllenCahn_SourceTerm_SOI", dims=2, family="reaction",
              reference="models/reaction/d2q9_AllenCahn_SourceTerm_SOI",
              description="D2Q9 Allen-Cahn advection-diffusion-reaction with second-order source integration")
    for k in range(9):
        px, py = k % 3, k // 3
        m.add_density(f"f[{k}]", CV[px], CV[py], 0, group="f", comment=f"LB density field f{px}{py}0")
    for n in ("Init_UX_External", "Init_UY_External", "Init_PhaseField_External"):
        m.add_density(n, 0, 0, 0, group="init", parameter=True)
    m.add_field("phaseField_tilde", stencil2d=1)
    m.add_global("PhaseFieldIntegral", comment="Total amount of phasefield", unit="1")
    m.add_quantity("PhaseField", unit="1")
    m.add_quantity("Q", unit="1")
    m.add_stage("InitFromFieldsStage", "InitFromFieldsStage", load_densities=True, save_fields=True)
    m.add_action("InitFromFields", ["InitFromFieldsStage"])
    m.add_node_type("DirichletEQ", "BOUNDARY")
    for n in ("SRT_DF_SOI", "SRT_M_SOI", "TRT_M_SOI", "TRT_CM_SOI"):
        m.add_node_type(n, "COLLISION")
    m.add_node_type("Wall", "BOUNDARY")
    S = m.add_setting
    S("diffusivity_phi", default=0.02, comment="Mobility")
    S("magic_parameter", default=0.25, comment="to control relaxation frequency of even moments in TRT collision kernel")
    S("lambda", default=1.0, comment="to control intensity of the source term")
    S("Init_UX", default=0, comment="free stream x-velocity", zonal=True)
    S("Init_UY", default=0, comment="free stream y-velocity", zonal=True)
    S("Init_PhaseField", zonal=True)
    S("CylinderCenterX_GH", default=0, comment="X coord of Gaussian Hill")
    S("CylinderCenterY_GH", default=0, comment="Y coord of Gaussian Hill")
    S("Sigma_GH", default=1, comment="Initial width of the Gaussian Hill", zonal=True)
    m.add_node_type("Smoothing", "ADDITIONALS")
    S("phase_field_smoothing_coeff", default=0)
    m.options = {"ExpotentialDecay": expdecay}
    m.set_dynamics("reaction/d2q9_AllenCahn_SourceTerm_SOI.inc")
    return m
