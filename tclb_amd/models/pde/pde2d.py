"""Finite-difference PDE models on the lattice runtime (reference models/PDE/*):
diffusion2D, advection_diffusion2D (option ``fields``), wave2D."""
from ..dsl import Model


def _common(m, field_names):
    for n in field_names:
        m.add_field(n, dx=(-1, 1), dy=(-1, 1))
    m.add_setting("Value", zonal=True)
    m.add_node_type("Dirichlet", "BOUNDARY")


def build_diffusion() -> Model:
    m = Model("diffusion2D", dims=2, family="PDE", reference="models/PDE/diffusion2D",
              description="explicit diffusion equation (5-point Laplacian)")
    _common(m, ["phi"])
    m.add_quantity("Phi")
    m.add_setting("diff_coeff")
    m.set_dynamics("pde/diffusion2D.inc")
    return m


def build_advection_diffusion(fields: bool = False) -> Model:
    m = Model("advection_diffusion2D", dims=2, family="PDE", reference="models/PDE/advection_diffusion2D",
              description="explicit advection-diffusion equation")
    _common(m, ["phi"])
    m.add_quantity("Phi")
    m.add_setting("diff_coeff")
    if fields:
        m.add_density("ux", 0, 0, 0, group="u", parameter=True, comment="free stream velocity")
        m.add_density("uy", 0, 0, 0, group="u", parameter=True, comment="free stream velocity")
        m.add_density("phi0", 0, 0, 0, group="init", parameter=True, comment="initial phi")
        m.add_stage("InitFromFieldsStage", "InitFromFields", load_densities=True, save_fields=True)
        m.add_action("InitFromFields", ["InitFromFieldsStage"])
    else:
        m.add_setting("ux", comment="free stream velocity")
        m.add_setting("uy", comment="free stream velocity")
    m.options = {"fields": fields}
    m.set_dynamics("pde/advection_diffusion2D.inc")
    return m


def build_wave(autosym: int = 0) -> Model:
    """reference OPT="autosym": symmetry node types mirror the u/v stencil reads"""
    m = Model("wave2D", dims=2, family="PDE", reference="models/PDE/wave2D",
              description="explicit damped wave equation")
    m.options["autosym"] = autosym
    _common(m, ["u", "v"])
    m.add_quantity("U")
    m.add_setting("Speed")
    m.add_setting("Viscosity")
    m.set_dynamics("pde/wave2D.inc")
    return m
