"""Model description DSL.

Python re-design of the reference's R model DSL (reference: src/conf.R:54-360).  A
model file builds a :class:`Model` with the same verbs the reference offers —
``add_density`` (AddDensity), ``add_field`` (AddField), ``add_setting`` (AddSetting),
``add_global`` (AddGlobal), ``add_quantity`` (AddQuantity), ``add_node_type``
(AddNodeType), ``add_stage``/``add_action`` (AddStage/AddAction) — plus the name of a
hand-written C++ dynamics include and optional sympy "codegen blocks".  The static
emitter (:mod:`tclb_amd.emit.emitter`) turns a Model into a per-model HIP/C++ header.

Derived tables (node-type bit packing, zone bits, ordering of globals, InObj
settings, the stage field-access hazard check) follow the reference's semantics:
node-type groups sorted by name get ceil(log2(n+1)) bits each, zone index in the
remaining high bits (src/conf.R:600-699); SUM globals first, then Objective, then
MAX globals (src/conf.R:740-751); every SUM global gets a zonal ``<G>InObj`` weight
(src/conf.R:753-761); stages may not read fields before they are written in an
action (src/conf.R:512-586).
"""
from __future__ import annotations

import os

import math
import re
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple



# models built with ADJOINT=1 in the reference (their conf.mk): they carry the Descent /
# GradientSmooth settings of the optimisation loop
ADJOINT_MODELS = {"d2q9_adj", "d2q9_optimalMixing", "d2q9_heat_adj", "d2q9_kuper_adj", "d3q19_heat_adj", "d3q19_adj",
                  "d2q9_plate", "sw", "d3q19_heat_adj_art", "d3q19_heat_adj_prop", "d2q9_diff"}

@dataclass
class Field:
    name: str                      # C++ member name (e.g. "f[3]" or "psi")
    group: str                     # group tag (stage load/save selection, VTK, checkpoints)
    index: int                     # index inside member array (-1: scalar member named `array`)
    nicename: str                  # identifier-safe name, e.g. f3
    stencil: Tuple[Tuple[int, int], Tuple[int, int], Tuple[int, int]] = ((0, 0), (0, 0), (0, 0))
    comment: str = ""
    parameter: bool = False
    average: bool = False
    default: float = 0.0
    shift: Optional[float] = None
    is_density: bool = False
    array: str = ""                # C++ member: array name (index >= 0) or scalar name

@dataclass
class Density:
    field: Field
    dx: int
    dy: int
    dz: int


@dataclass
class Setting:
    name: str
    default: float = 0.0
    unit: str = "1"
    zonal: bool = False
    derived: Dict[str, str] = field(default_factory=dict)   # target setting -> expression
    comment: str = ""
    preload: bool = True
    default_str: Optional[str] = None                       # default with units ("0m/s")


@dataclass
class Global:
    name: str
    unit: str = "1"
    op: str = "SUM"
    comment: str = ""


@dataclass
class Quantity:
    name: str
    unit: str = "1"
    vector: bool = False
    comment: str = ""
    adjoint: bool = False          # computed from the adjoint state (reference adjoint=T)
    adjoint_of: Optional[str] = None   # field or density group whose adjoint it reports


@dataclass
class NodeType:
    name: str
    group: str
    value: int = 0
    mask: int = 0
    shift: int = 0


@dataclass
class Stage:
    name: str
    main: str
    load_densities: bool = True
    save_fields: Optional[List[str]] = None   # nicenames; None = all fields
    read_fields: Optional[List[str]] = None   # nicenames read with stencil (for hazard check)
    fixed_point: bool = False
    snapshot_reads: bool = False   # reads of its own saved fields see the pre-stage values
    particle: bool = False
    init: bool = False                        # "Init" stream: no load before main
    lazy_load: bool = False   # the declared loads are not made before main: main calls
                              # load_<name>() where it needs them (declared for the halo)
    lds: Optional[List[str]] = None   # fields read through a stencil that the GPU kernel
                                      # stages in LDS tiles (executor_hip.hpp k_tile)
    split: bool = False       # GPU: two kernels by node class (Node::node_class_(): 1 =
                              # the common interior path, 2 = the rest), each compiled with
                              # its own path only and so its own register budget
    defer: bool = False       # split stage whose class-1 path hands the nodes that need a
                              # rare heavy branch to a third kernel (Node::defer_heavy)
    keep: Optional[List[str]] = None   # fields (nicenames / group tags) the stage leaves
                                       # unchanged and does not store; the lattice keeps
                                       # both snapshots' copies equal (Lattice._mirror_kept)


@dataclass
class Action:
    name: str
    stages: List[str]


class ModelError(Exception):
    pass


_ident = re.compile(r"[^A-Za-z0-9_]")


def nicename(name: str) -> str:
    return _ident.sub("", name)


class Model:
    def __init__(self, name: str, dims: int = 3, family: str = "", description: str = "",
                 reference: str = ""):
        self.name = name
        self.dims = dims
        self.family = family
        self.description = description
        self.reference = reference     # reference model directory (parity pointer)
        self.fields: List[Field] = []
        self.densities: List[Density] = []
        self.settings: List[Setting] = []
        self.globals_: List[Global] = []
        self.quantities: List[Quantity] = []
        self.node_types: List[NodeType] = []
        self.stages: List[Stage] = []
        self.actions: List[Action] = []
        self.options: Dict[str, bool] = {}
        self.dynamics: Optional[str] = None          # include path (relative to csrc/models)
        self.codegen_blocks: List[Callable[["Model"], str]] = []
        # hand-written reverse-mode node adjoints: stage main -> (predicate, function)
        # member names in the dynamics (see set_reverse)
        self.reverse: Dict[str, tuple] = {}
        # kept fields whose value is a global setting (or a constant) on every node: the
        # lattice fills them on both snapshots instead of copying them (setting_fields)
        self.setting_fields: Dict[str, object] = {}
        self.color: Optional[tuple] = None     # (value, weight) C++ expressions of Color()
        # waves/SIMD floor of the globals-integrating stage kernels (0: compiler's choice);
        # see executor_hip.hpp k_stage_glob
        self.glob_waves: int = 2
        self.lattices: Dict[str, str] = {}           # group -> lattice name (weights table)
        self.defines: Dict[str, str] = {}
        self.objectives: Dict[str, str] = {}        # AddObjective: name -> expression of globals
        self._finalized = False

    # ------------------------------------------------------------------ verbs
    def _split_name(self, name: str, group: Optional[str]):
        m = re.match(r"^([A-Za-z_][A-Za-z0-9_]*)\[(\d+)\]$", name)
        if m:
            return m.group(1), int(m.group(2))
        return (group or name), None

    def add_density(self, name: str, dx: int = 0, dy: int = 0, dz: int = 0, group: Optional[str] = None,
                    parameter: bool = False, average: bool = False, default: float = 0.0,
                    shift: Optional[float] = None, comment: str = ""):
        """AddDensity (src/conf.R:65-102): a streamed population, pulled from (-dx,-dy,-dz)."""
        arr, idx = self._split_name(name, None)
        grp = group if group is not None else arr
        if idx is None:
            arr, idx = name, -1
        f = Field(name=name, group=grp, index=idx, nicename=nicename(name), array=arr,
                  stencil=((min(0, -dx), max(0, -dx)), (min(0, -dy), max(0, -dy)), (min(0, -dz), max(0, -dz))),
                  comment=comment, parameter=parameter, average=average, default=default, shift=shift,
                  is_density=True)
        self._add_field(f)
        self.densities.append(Density(field=f, dx=dx, dy=dy, dz=dz))
        return f

    def add_densities(self, group: str, vectors: Sequence[Sequence[int]], names: Optional[Sequence[str]] = None,
                      **kw):
        out = []
        for i, v in enumerate(vectors):
            v = list(v) + [0] * (3 - len(v))
            nm = names[i] if names else f"{group}[{i}]"
            out.append(self.add_density(nm, v[0], v[1], v[2], group=group, **kw))
        return out

    def add_field(self, name: str, dx=(0, 0), dy=(0, 0), dz=(0, 0), stencil2d: Optional[int] = None,
                  stencil3d: Optional[int] = None, group: Optional[str] = None, comment: str = "",
                  parameter: bool = False, average: bool = False, default: float = 0.0):
        """AddField (src/conf.R:135-176): stored per-node array readable with a stencil."""
        def rng(v):
            if isinstance(v, int):
                return (min(0, v), max(0, v))
            return (min(v), max(v))
        sx, sy, sz = rng(dx), rng(dy), rng(dz)
        if stencil2d is not None:
            sx = (-stencil2d, stencil2d); sy = (-stencil2d, stencil2d)
        if stencil3d is not None:
            sx = (-stencil3d, stencil3d); sy = (-stencil3d, stencil3d); sz = (-stencil3d, stencil3d)
        existing = [f for f in self.fields if f.name == name]
        if existing:
            f = existing[0]
            f.stencil = ((min(f.stencil[0][0], sx[0]), max(f.stencil[0][1], sx[1])),
                         (min(f.stencil[1][0], sy[0]), max(f.stencil[1][1], sy[1])),
                         (min(f.stencil[2][0], sz[0]), max(f.stencil[2][1], sz[1])))
            return f
        arr, idx = self._split_name(name, None)
        if idx is None:
            arr, idx = name, -1
        f = Field(name=name, group=group or arr, index=idx, nicename=nicename(name), array=arr,
                  stencil=(sx, sy, sz), comment=comment, parameter=parameter, average=average, default=default)
        self._add_field(f)
        return f

    def _add_field(self, f: Field):
        if any(g.nicename == f.nicename for g in self.fields):
            raise ModelError(f"duplicate field {f.name} in model {self.name}")
        self.fields.append(f)

    def add_setting(self, name: str, default=0.0, unit: str = "1", zonal: bool = False, comment: str = "",
                    derived: Optional[Dict[str, str]] = None, preload: bool = True, **derived_kw):
        """AddSetting (src/conf.R:179-214).  ``derived_kw`` mirrors the reference's
        ``AddSetting(name="nu", omega='1.0/(3*nu+0.5)')`` form."""
        dv = dict(derived or {})
        dv.update({k: v for k, v in derived_kw.items() if isinstance(v, str)})
        dstr = None
        if isinstance(default, str):
            dstr = default
            m = re.match(r"^\s*([-+0-9.eE]+)", default)
            default = float(m.group(1)) if m else 0.0
        for s in self.settings:
            if s.name == name:
                s.derived.update(dv)
                return s
        s = Setting(name=name, default=float(default), unit=unit, zonal=zonal, derived=dv, comment=comment,
                    preload=preload, default_str=dstr)
        self.settings.append(s)
        return s

    def add_global(self, name: str, unit: str = "1", op: str = "SUM", comment: str = ""):
        """AddGlobal (src/conf.R:217-235)."""
        if op not in ("SUM", "MAX"):
            raise ModelError(f"unknown global op {op}")
        g = Global(name=name, unit=unit, op=op, comment=comment)
        self.globals_.append(g)
        return g

    def add_quantity(self, name: str, unit: str = "1", vector: bool = False, comment: str = "",
                     adjoint: bool = False, adjoint_of: Optional[str] = None):
        """AddQuantity (src/conf.R:237-257): requires get<name>() in the dynamics, except
        for adjoint quantities (``adjoint=True``, reference AddQuantity(adjoint=T)), which
        the runtime derives from the last adjoint sweep: ``<F>B`` is dJ/d(field F),
        ``RhoB`` the sum over the adjoint populations of the first density group;
        ``adjoint_of`` names the field (its adjoint) or density group (sum of adjoints)."""
        q = Quantity(name=name, unit=unit, vector=vector, comment=comment, adjoint=adjoint,
                     adjoint_of=adjoint_of)
        self.quantities.append(q)
        return q

    def add_objective(self, name: str, expr: str):
        """AddObjective (src/conf.R:349-360): a named objective function of the globals
        (sympy-parsable expression), selectable as an attribute of <Objective>."""
        self.objectives[name] = expr

    def add_node_type(self, name: str, group: str):
        """AddNodeType (src/conf.R:259-270)."""
        if any(n.name == name for n in self.node_types):
            return
        self.node_types.append(NodeType(name=name, group=group))

    def add_stage(self, name: str, main: Optional[str] = None, load_densities=False,
                  save_fields=False, read_fields: Optional[Sequence[str]] = None,
                  fixed_point: bool = False, particle: bool = False, init: bool = False,
                  snapshot_reads: bool = False, lazy_load: bool = False, lds: Optional[Sequence[str]] = None,
                  split: bool = False, keep: Optional[Sequence[str]] = None, defer: bool = False):
        """AddStage (src/conf.R:295-330): load_densities / save_fields are True (all), False
        (none) or lists of field names / group tags (reference defaults: FALSE).
        lazy_load: the stage's main pulls its densities itself (load_<name>()), e.g. only
        on the nodes a particle covers; the loads still count for halos and hazards.
        lds: fields (nicenames) the stage reads through a stencil, staged in LDS tiles by the
        GPU kernel (no reference counterpart: a MI355X schedule hint; the node code is
        unchanged, the CPU and AD executors ignore it).
        split: the GPU runs the stage as two kernels over the same box, one per node class
        (the node code's node_class_(); its CLS_ template argument is 1 / 2 in them, 0 in
        the executors that run every node in one pass), so a rare heavy path (boundary
        closures) does not set the register budget, and with it the occupancy, of the
        common one.
        defer: (split stages) the class-1 node code may hand a node to a third kernel at
        run time: defer_heavy(cond) is true, in the class-1 kernel, where the node needs the
        heavy branch — the node is then not stored and its tile is queued — and, in that
        third kernel (CLS_ 3, over the queued tiles only, no globals), where it does not.
        So a heavy branch that depends on field values (e.g. a media interface that moves
        with the particles) also leaves the common kernel's register budget.  Globals must
        be added before the defer point.  The node code also defines defer_pre_(stage): the
        same test from what the node can read before the stage's loads (true when unsure),
        which the CLS_ 3 kernel runs first.  CPU and unsplit executors: never defers.
        keep: entries of save_fields (same tags) that the stage never changes, e.g. wall
        normals set at initialisation: they are not stored (no read and write of them per
        node and step) and the lattice copies them into the other snapshot once before an
        action that has such a stage runs (no reference counterpart: TCLB stores every
        declared field in every step)."""
        if save_fields is True:
            save_fields = None
        elif save_fields is False:
            save_fields = []
        if keep:
            if save_fields is None or any(k not in save_fields for k in keep):
                raise ModelError(f"stage {name}: keep entries must be entries of an explicit save_fields list")
            save_fields = [x for x in save_fields if x not in keep]
        st = Stage(name=name, main=main or name, load_densities=load_densities,
                   save_fields=list(save_fields) if save_fields is not None else None,
                   read_fields=list(read_fields) if read_fields is not None else None,
                   fixed_point=fixed_point, particle=particle, init=init, snapshot_reads=snapshot_reads,
                   lazy_load=lazy_load, lds=list(lds) if lds else None, split=split,
                   keep=list(keep) if keep else None, defer=defer)
        if defer and not split:
            raise ModelError(f"stage {name}: defer needs split=True")
        self.stages = [s for s in self.stages if s.name != name] + [st]
        return st

    def add_action(self, name: str, stages: Sequence[str]):
        """AddAction (src/conf.R:331-345)."""
        self.actions = [a for a in self.actions if a.name != name] + [Action(name=name, stages=list(stages))]

    def set_dynamics(self, include: str):
        self.dynamics = include

    def set_reverse(self, stage_main: str, predicate: str, function: str):
        """reverse-mode adjoint of the stages running ``stage_main``: on nodes where the
        dynamics' ``predicate()`` holds, the AD executors call ``function(const AdCtx&)``
        (one reverse sweep of the node: transposed Jacobian-vector product pushed to the
        load sites) instead of the forward-mode dual-number passes; the reference gets
        its reverse sweep from Tapenade (tools/makeAD)"""
        self.reverse[stage_main] = (predicate, function)

    def set_color(self, value: str, weight: str = "1"):
        """the node colour of the frame renderer (reference ``Color()``: a value mapped
        through the colour scale and a weight, 0 drawing the node green), as C++
        expressions of the node; the default is |U| and 0 on Solid nodes"""
        self.color = (value, weight)

    def add_codegen(self, fn: Callable[["Model"], str]):
        self.codegen_blocks.append(fn)

    # ------------------------------------------------------------ derivation
    def finalize(self):
        if self._finalized:
            return self
        # default stages/actions (src/conf.R:459-472)
        if not any(s.name == "BaseIteration" for s in self.stages):
            self.stages.insert(0, Stage(name="BaseIteration", main="Run"))
        if not any(s.name == "BaseInit" for s in self.stages):
            self.stages.insert(1, Stage(name="BaseInit", main="Init", load_densities=False, init=True))
        if not any(a.name == "Iteration" for a in self.actions):
            self.actions.insert(0, Action("Iteration", ["BaseIteration"]))
        if not any(a.name == "Init" for a in self.actions):
            self.actions.insert(1, Action("Init", ["BaseInit"]))
        # globals ordering: SUM, Objective, MAX (src/conf.R:740-751)
        self.globals_ = [g for g in self.globals_ if g.name != "Objective"]
        sums = [g for g in self.globals_ if g.op == "SUM"]
        maxs = [g for g in self.globals_ if g.op != "SUM"]
        self.globals_ = sums + [Global("Objective", comment="Objective function")] + maxs
        self.n_sum_globals = len(sums) + 1
        for g in sums:
            self.add_setting(f"{g.name}InObj", default=0.0, zonal=True,
                             comment=f"Weight of [{g.comment or g.name}] in objective", preload=False)
        self.add_setting("Threshold", default=0.5, comment="Parameters threshold")
        if os.path.basename(self.reference or self.name) in ADJOINT_MODELS:
            # reference src/conf.R:725-738 (ADJOINT=1 models only)
            if self.setting("Descent") is None:
                self.add_setting("Descent", default=0.0, comment="Optimization Descent")
            if self.setting("GradientSmooth") is None:
                self.add_setting("GradientSmooth", default=0.0, comment="Gradient smoothing in OptSolve")
        autosym = int(self.options.get("autosym", 0) or 0)
        if autosym:   # automatic symmetry node types (src/conf.R:440-457)
            nm = "Symmetry" if autosym == 1 else "SymmetryEdge"
            for ax in ("X", "Y", "Z")[:max(2, self.dims)]:
                self.add_node_type(f"{nm}{ax}_plus", f"SYM{ax}")
                self.add_node_type(f"{nm}{ax}_minus", f"SYM{ax}")
        self._pack_node_types()
        self._check_stage_access()
        self._check_lds()
        self._finalized = True
        return self

    def _pack_node_types(self):
        shift_num = 0
        groups: Dict[str, List[NodeType]] = {}
        for n in self.node_types:
            groups.setdefault(n.group, []).append(n)
        self.group_masks: Dict[str, int] = {}
        self.group_shift: Dict[str, int] = {}
        for gname in sorted(groups):
            tab = groups[gname]
            n = len(tab)
            bits = int(math.ceil(math.log2(n + 1)))
            for i, nt in enumerate(tab):
                nt.value = (1 << shift_num) * (i + 1)
                nt.mask = (1 << shift_num) * ((1 << bits) - 1)
                nt.shift = shift_num
            self.group_masks[gname] = (1 << shift_num) * ((1 << bits) - 1)
            self.group_shift[gname] = shift_num
            shift_num += bits
        self.flag_bits = 16 if shift_num <= 14 else 32
        if shift_num > 30:
            raise ModelError("NodeTypes exceed 32 bits")
        self.zone_shift = shift_num
        self.zone_bits = self.flag_bits - shift_num
        self.zone_max = (1 << self.zone_bits) - 1
        self.group_masks["SETTINGZONE"] = self.zone_max << shift_num
        self.group_shift["SETTINGZONE"] = shift_num
        self.group_masks["NONE"] = 0
        self.group_masks["ALL"] = (1 << self.flag_bits) - 1

    def _check_stage_access(self):
        """Static field-access hazard check (reference: src/conf.R:512-586)."""
        names = {f.nicename for f in self.fields}
        for act in self.actions:
            written: set = set()
            for sname in act.stages:
                st = self.stage(sname)
                if st is None:
                    raise ModelError(f"action {act.name} references unknown stage {sname}")
                reads = set(st.read_fields or [])
                bad = reads - names
                if bad:
                    raise ModelError(f"stage {st.name} reads unknown fields {sorted(bad)}")
                saves = {f.nicename for f in self.fields if self.matches(f, st.save_fields)}
                overl = reads & saves
                if overl and not st.init and st.read_fields is not None:
                    # reading a field with a stencil while writing it in the same stage is a race
                    nonlocal_reads = [f for f in overl if self.field(f).stencil != ((0, 0), (0, 0), (0, 0))]
                    if nonlocal_reads:
                        raise ModelError(f"stage {st.name} reads and writes {sorted(nonlocal_reads)} "
                                         f"with a stencil (data race)")
                written |= saves

    def _check_lds(self):
        """LDS-staged fields of a stage: existing, not written by the stage (a tile is a
        read-only copy of the input snapshot), stencil at most 2 nodes deep"""
        for st in self.stages:
            for name in st.lds or []:
                f = self.field(name)
                if f is None:
                    raise ModelError(f"stage {st.name}: lds field {name} does not exist")
                if self.matches(f, st.save_fields):
                    raise ModelError(f"stage {st.name}: lds field {name} is written by the stage")
                if max(max(-a, b) for a, b in f.stencil) > 2:
                    raise ModelError(f"stage {st.name}: lds field {name} has a stencil deeper than 2")

    def late_reads(self, action: str) -> List[str]:
        """fields that a stage k > 0 of `action` reads (declared reads, loaded densities)
        although no earlier stage of the action wrote them: such a stage sees what the
        output snapshot held before the step, i.e. the state of two steps back (the
        reference rejects these unless its access check is permissive, src/conf.R:512-586)"""
        act = self.action(action)
        if act is None:
            return []
        written: set = set()
        out: set = set()
        for k, sname in enumerate(act.stages):
            st = self.stage(sname)
            if k > 0:
                reads = set(st.read_fields or [])
                if st.load_densities and not st.init:
                    reads |= {d.field.nicename for d in self.densities if self.matches(d.field, st.load_densities)}
                out |= reads - written
            written |= {f.nicename for f in self.fields if self.matches(f, st.save_fields)}
        return sorted(out)

    # ---------------------------------------------------------------- lookup
    def stage(self, name: str) -> Optional[Stage]:
        for s in self.stages:
            if s.name == name:
                return s
        return None

    def stage_index(self, name: str) -> int:
        for i, s in enumerate(self.stages):
            if s.name == name:
                return i
        raise KeyError(name)

    def action(self, name: str) -> Optional[Action]:
        for a in self.actions:
            if a.name == name:
                return a
        return None

    def field(self, nice: str) -> Field:
        for f in self.fields:
            if f.nicename == nice or f.name == nice:
                return f
        raise KeyError(nice)

    def field_index(self, nice: str) -> int:
        for i, f in enumerate(self.fields):
            if f.nicename == nice or f.name == nice:
                return i
        raise KeyError(nice)

    @property
    def global_settings(self) -> List[Setting]:
        return [s for s in self.settings if not s.zonal]

    @property
    def zonal_settings(self) -> List[Setting]:
        return [s for s in self.settings if s.zonal]

    def setting(self, name: str) -> Optional[Setting]:
        for s in self.settings:
            if s.name == name:
                return s
        return None

    def node_type(self, name: str) -> Optional[NodeType]:
        for n in self.node_types:
            if n.name == name:
                return n
        return None

    def group_arrays(self) -> Dict[str, int]:
        """C++ members: array name -> size (scalar members have size 0)."""
        out: Dict[str, int] = {}
        for f in self.fields:
            if f.index >= 0:
                out[f.array] = max(out.get(f.array, 0), f.index + 1)
            else:
                out.setdefault(f.array, 0)
        return out

    def matches(self, f: Field, spec) -> bool:
        """stage load/save selection: True/None = all, False = none, list of names/groups"""
        if spec is None or spec is True:
            return True
        if spec is False:
            return False
        return f.name in spec or f.nicename in spec or f.group in spec

    def halo(self) -> Tuple[int, int, int]:
        """max |stencil| per axis (reference BorderMargin, src/conf.R:1017-1023)."""
        hx = max([max(-f.stencil[0][0], f.stencil[0][1]) for f in self.fields] + [0])
        hy = max([max(-f.stencil[1][0], f.stencil[1][1]) for f in self.fields] + [0])
        hz = max([max(-f.stencil[2][0], f.stencil[2][1]) for f in self.fields] + [0])
        return hx, hy, hz

    def describe(self) -> str:
        self.finalize()
        lines = [f"Model {self.name} ({self.dims}D, family {self.family})", self.description, ""]
        lines.append(f"Fields ({len(self.fields)}): " + ", ".join(f.name for f in self.fields))
        lines.append("Settings: " + ", ".join(f"{s.name}{'[zonal]' if s.zonal else ''}={s.default}"
                                              for s in self.settings))
        lines.append("Globals: " + ", ".join(f"{g.name}({g.op})" for g in self.globals_))
        lines.append("Quantities: " + ", ".join(q.name + ("[vec]" if q.vector else "") for q in self.quantities))
        lines.append("Node types: " + ", ".join(f"{n.name}<{n.group}>={n.value:#x}" for n in self.node_types))
        lines.append("Stages: " + ", ".join(f"{s.name}:{s.main}" for s in self.stages))
        lines.append("Actions: " + ", ".join(f"{a.name}=[{','.join(a.stages)}]" for a in self.actions))
        return "\n".join(lines)
