"""d2q9_ShanChen — single-component pseudopotential (Shan-Chen) multiphase model with
solid-fluid adhesion; two-stage iteration (BaseIteration + PsiIteration).
Reference: models/multiphase/d2q9_ShanChen/Dynamics.R, Dynamics.c.Rt."""
from ..dsl import Model

U9 = [[0, 0], [1, 0], [0, 1], [-1, 0], [0, -1], [1, 1], [-1, 1], [-1, -1], [1, -1]]


def build() -> Model:
    m = Model("d2q9_ShanChen", dims=2, family="multiphase", reference="models/multiphase/d2q9_ShanChen",
              description="D2Q9 Shan-Chen pseudopotential multiphase (psi = 1 - exp(-rho))")
    for i, (x, y) in enumerate(U9):
        m.add_density(f"f[{i}]", x, y, 0, group="f")
    m.add_density("rho", 0, 0, 0, group="density")
    m.add_field("psi", stencil2d=1, group="pp")
    m.add_field("neighbour_type", stencil2d=1, group="neighbour_type_group")
    m.add_stage("BaseInit", "Init", save_fields=["f", "density", "neighbour_type_group"], load_densities=["f", "density"])
    # the interaction force reads psi through a stencil: staged in LDS tiles on the GPU
    m.add_stage("BaseIteration", "Run", save_fields=["f", "density", "neighbour_type_group"],
                load_densities=["f", "density", "neighbour_type_group"], lds=["psi"])
    m.add_stage("PsiIteration", "calcPsi", save_fields=["psi"], load_densities=["f", "density"])
    m.add_action("Init", ["BaseInit", "PsiIteration"])
    m.add_action("Iteration", ["BaseIteration", "PsiIteration"])
    m.add_quantity("U", unit="m/s", vector=True)
    m.add_quantity("Rho", unit="kg/m3")
    m.add_quantity("Psi", unit="1")
    m.add_setting("omega", comment="inverse of relaxation time")
    m.add_setting("viscosity", default=0.16666666, comment="kinematic viscosity", omega="1.0/(3*viscosity+0.5)")
    m.add_setting("VelocityX", default=0, comment="inlet/outlet/init velocity", zonal=True)
    m.add_setting("VelocityY", default=0, comment="inlet/outlet/init velocity", zonal=True)
    m.add_setting("GravitationX", default=0, comment="body/external acceleration", zonal=True)
    m.add_setting("GravitationY", default=0, comment="body/external acceleration", zonal=True)
    m.add_setting("Density", default=1, comment="Density", zonal=True)
    m.add_node_type("MovingWall", "BOUNDARY")
    m.add_setting("G_ff", default=0, comment="fluid-fluid interaction strength")
    m.add_setting("G_sf", default=0, comment="solid-fluid interaction strength")
    m.add_node_type("Solid", "BOUNDARY")
    m.add_node_type("Wall", "BOUNDARY")
    m.add_node_type("MRT", "COLLISION")
    m.set_dynamics("multiphase/d2q9_shanchen.inc")
    return m
