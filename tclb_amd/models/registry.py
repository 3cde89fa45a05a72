"""Model registry (replaces the reference's conf.mk discovery, src/models.R:20-90).

Every model is a Python module exposing ``build() -> Model``; variants (the reference's
``OPT=`` option products, e.g. ``d2q9_bc_autosym``) are registered as separate entries
with option dictionaries."""
from __future__ import annotations

import importlib
from typing import Callable, Dict, List, Optional

from .dsl import Model

# name -> (module, kwargs)
_MODELS: Dict[str, tuple] = {}


def register(name: str, module: str, builder: str = "build", **kwargs):
    _MODELS[name] = (module, builder, kwargs)


def names() -> List[str]:
    return sorted(_MODELS)


_cache: Dict[str, Model] = {}


def get(name: str) -> Model:
    if name not in _MODELS:
        raise KeyError(f"unknown model '{name}'; known: {', '.join(names())}")
    if name not in _cache:
        mod, builder, kw = _MODELS[name]
        m = importlib.import_module(mod, package=__package__)
        model = getattr(m, builder)(**kw)
        if model.name != name:
            model.name = name
        model.finalize()
        _cache[name] = model
    return _cache[name]


# ---- catalog ---------------------------------------------------------------------
register("d3q27", ".flow.d3q27")
register("d2q9", ".flow.d2q9")
register("d3q19", ".flow.d3q19")
register("d2q9_SRT", ".flow.d2q9_srt")
register("d2q9_ShanChen", ".multiphase.d2q9_shanchen")
register("diffusion2D", ".pde.pde2d", "build_diffusion")
register("advection_diffusion2D", ".pde.pde2d", "build_advection_diffusion")
register("advection_diffusion2D_fields", ".pde.pde2d", "build_advection_diffusion", fields=True)
register("wave2D", ".pde.pde2d", "build_wave")
register("d3q27_cumulant", ".flow.d3q27_cumulant")
register("d3q27_cumulant_qibb_small", ".flow.d3q27_cumulant_qibb_small")
register("d3q27_cumulant_AVG_IB_SMAG", ".flow.d3q27_cumulant", avg=True, ib=True, smag=True)
register("d3q19_heat", ".heat.d3q19_heat")
register("auto", ".flow.auto")
register("auto_d3q19", ".flow.auto", q19=True)
register("auto_d3q19_BGK", ".flow.auto", q19=True, coll="BGK")
register("auto_d3q19_TRT", ".flow.auto", q19=True, coll="TRT")
register("auto_d3q19_part", ".flow.auto", q19=True, part=True)
register("auto_d3q19_part_BGK", ".flow.auto", q19=True, part=True, coll="BGK")
register("auto_d3q19_part_TRT", ".flow.auto", q19=True, part=True, coll="TRT")
register("auto_part", ".flow.auto", part=True)
register("auto_BGK", ".flow.auto", coll="BGK")
register("auto_TRT", ".flow.auto", coll="TRT")
register("d3q19_les", ".flow.d3q19_les")
register("d3q27_pf_velocity", ".multiphase.d3q27_pf_velocity")
register("d3q27_pf_velocity_q27", ".multiphase.d3q27_pf_velocity", q27=True)
register("d3q27_pf_velocity_BGK", ".multiphase.d3q27_pf_velocity", bgk=True)
register("d2q9_bc", ".flow.d2q9", bc=True)
register("d2q9_autosym", ".flow.d2q9", autosym=1)
register("d2q9_bc_autosym", ".flow.d2q9", bc=True, autosym=1)
register("d2q9_kuper", ".multiphase.d2q9_kuper")
register("d2q9_pf", ".multiphase.d2q9_pf")
register("d2q9_pf_no_bc", ".multiphase.d2q9_pf", no_bc=True)
register("d2q9_pf_fd", ".multiphase.d2q9_pf", fd=True)
register("d2q9_npe_guo", ".electrokinetic.d2q9_npe_guo")
register("d2q9_thin_film", ".flow.d2q9_thin_film")
register("d3q27_PSM", ".particles.d3q27_psm")
register("d3q27_PSM_NEBB", ".particles.d3q27_psm", nebb=True)
register("d3q27_PSM_SUP", ".particles.d3q27_psm", sup=True)
register("d3q27_PSM_TRT_NEBB", ".particles.d3q27_psm", trt=True, nebb=True)
register("d3q27_PSM_MS_NEBB", ".particles.d3q27_psm", ms=True, nebb=True)
register("d3q27_PSM_KL_NEBB", ".particles.d3q27_psm", kl=True, nebb=True)
register("d3q27_PSM_NEBB_singlekernel", ".particles.d3q27_psm", nebb=True, singlekernel=True)
register("d2q9_adj", ".optimization.d2q9_adj")
register("d2q9_poison_boltzmann", ".electrokinetic.d2q9_poison_boltzmann")
register("d2q9_cumulant", ".flow.d2q9_cumulant")
register("d2q9_les", ".flow.d2q9_les")
register("d2q9_par", ".flow.d2q9", par=True)
register("d2q9_par_BC", ".flow.d2q9", par=True, bc=True)
register("d2q9_part", ".flow.d2q9", part=True)
register("d2q9_part_BC", ".flow.d2q9", part=True, bc=True)
register("d3q27_cumulant_part", ".flow.d3q27_cumulant", part=True)
register("d3q27_cumulant_part_AVG_IB_SMAG", ".flow.d3q27_cumulant", part=True, avg=True, ib=True, smag=True)
register("d3q27_BGK", ".flow.d3q27_bgk")
register("d3q27_BGK_galcor", ".flow.d3q27_bgk", galcor=True)
register("d3q19_kuper", ".multiphase.d3q19_kuper")
register("d3q27_kl", ".nonnewtonian.d3q27_kl")
register("d3q27_kl_OutFlow", ".nonnewtonian.d3q27_kl", outflow=True)
register("d3q27_viscoplastic", ".nonnewtonian.d3q27_viscoplastic")
register("d3q27_viscoplastic_OutFlow", ".nonnewtonian.d3q27_viscoplastic", outflow=True)
register("d2q9_diff", ".experimental.d2q9_diff")
register("d2q9_lbmpy", ".flow.d2q9_lbmpy")
register("d2q9_optimalMixing", ".optimization.d2q9_optimalmixing")
register("d2q9_heat", ".heat.d2q9_heat")
register("d3q19_adj", ".optimization.d3q19_adj")
register("d3q19_heat_adj", ".optimization.d3q19_heat_adj")
register("d3q19_heat_adj_art", ".optimization.d3q19_heat_adj_art")
register("d3q19_heat_adj_prop", ".optimization.d3q19_heat_adj_prop")
register("sw", ".shallowwater.sw")
register("d2q9_plate", ".moving.d2q9_plate")
register("d2q9_inc", ".experimental.d2q9_inc")
register("d2q9_heat_adj", ".optimization.d2q9_heat_adj")
register("d2q9_solid", ".multiphase.d2q9_solid")
for _sys in ("AllenCahn", "SIR_SimpleLaplace", "SIR_ModifiedPeng", "SimpleDiffusion", "LinearReaction"):
    register(f"d2q9_reaction_diffusion_system_{_sys}", ".reaction.d2q9_reaction_diffusion_system", system=_sys)
    for _opt, _int in (("Trapezoidal", "Trapezoid"), ("Midpoint", "Midpoint"), ("Heun", "Heun"), ("Euler", "Euler")):
        register(f"d2q9_reaction_diffusion_system_{_sys}_{_opt}", ".reaction.d2q9_reaction_diffusion_system",
                 system=_sys, integrator=_int)
register("d2q9_lee", ".multiphase.d2q9_lee")
register("d2q9_pp_LBL", ".multiphase.d2q9_pp_LBL")
register("d2q9_pp_MCMP", ".multiphase.d2q9_pp_MCMP")
register("d2q9_hb", ".experimental.d2q9_hb")
register("d2q9_pf_pressureEvolution", ".multiphase.d2q9_pf_pressureEvolution")
register("d2q9_AllenCahn_SourceTerm_SOI", ".reaction.d2q9_AllenCahn_SourceTerm_SOI")
register("d2q9_AllenCahn_SourceTerm_SOI_ExpotentialDecay", ".reaction.d2q9_AllenCahn_SourceTerm_SOI", expdecay=True)
register("d2q9_kuper_adj", ".optimization.d2q9_kuper_adj")
register("d2q9_pf_velocity", ".multiphase.d2q9_pf_velocity")
for _o in ("GF", "RT", "Outflow", "GuoCM", "debug", "BGK", "CM"):
    register(f"d2q9_pf_velocity_{_o}", ".multiphase.d2q9_pf_velocity", **{_o.lower(): True})
register("d2q9_pf_velocity_autosym", ".multiphase.d2q9_pf_velocity", autosym=1)
register("d3q27_cumulant_heat", ".heat.d3q27_cumulant_heat")
register("d2q9q9_cm_cht", ".heat.d2q9q9_cm_cht")
for _o in ("OutFlowConvective", "OutFlowNeumann", "AVG", "IBB", "SMAG", "CHT"):
    register(f"d2q9q9_cm_cht_{_o}", ".heat.d2q9q9_cm_cht", **{_o.lower(): True})
register("d3q27q7_cm_cht", ".heat.d3q27q7_cm_cht")
for _o in ("OutFlowConvective", "OutFlowNeumann", "AVG", "IBB", "SMAG", "CHT"):
    register(f"d3q27q7_cm_cht_{_o}", ".heat.d3q27q7_cm_cht", **{_o.lower(): True})
register("d3q27q27_cm_cht", ".heat.d3q27q7_cm_cht", heat_q=27)
for _o in ("OutFlowConvective", "OutFlowNeumann", "AVG", "IBB", "SMAG", "CHT"):
    register(f"d3q27q27_cm_cht_{_o}", ".heat.d3q27q7_cm_cht", heat_q=27, **{_o.lower(): True})
