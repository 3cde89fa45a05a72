"""Handler framework: XML element -> behaviour object.

Mirrors the reference control layer (reference: src/Handlers/vHandler.h:33-104,
src/Handlers.h:12-85, src/Factory.h:20-74): handler kinds CALLBACK / ACTION / DESIGN /
GENERIC / CONTAINER, scheduling by ``Iterations`` (Now/Next/Prev with a start
iteration), a registry keyed by element name, and ``GenericAction.execute_internal``
which stacks periodic callbacks and designs on ``solver.hands`` and runs one-shot
callbacks immediately (src/Handlers/GenericAction.cpp:10-56).
"""
from __future__ import annotations

import math
import xml.etree.ElementTree as ET
from typing import Dict, Optional, Type

from ..utils.log import log

HANDLER_CALLBACK = 0x01
HANDLER_ACTION = 0x02
HANDLER_DESIGN = 0x04
HANDLER_GENERIC = 0x10
HANDLER_CONTAINER = 0x20

ITERATION_STOP = 1

REGISTRY: Dict[str, Type["Handler"]] = {}


def register(*names):
    def deco(cls):
        for n in names:
            REGISTRY[n] = cls
        return cls
    return deco


class HandlerError(RuntimeError):
    pass


class Handler:
    kind = HANDLER_GENERIC

    def __init__(self, node: ET.Element, solver):
        self.node = node
        self.solver = solver
        self.start_iter = 0
        self.every_iter = 0.0

    # -- attribute helpers --------------------------------------------------------
    def attr(self, name: str, default=None):
        return self.node.get(name, default)

    def context_attr(self, name: str, default=None):
        """reference vHandler::context_attribute: nearest ancestor-or-self attribute"""
        n = self.node
        parents = getattr(self.solver, "_xml_parents", {})
        while n is not None:
            if n.get(name) is not None:
                return n.get(name)
            n = parents.get(n)
        return default

    def alt(self, name: str, default=None):
        v = self.node.get(name)
        if v is None:
            return default
        return self.solver.units.alt(v)

    # -- lifecycle ----------------------------------------------------------------
    def init(self) -> int:
        return 0

    def do_it(self) -> int:
        return 0

    def finish(self) -> int:
        return 0

    # -- scheduling (reference vHandler::Now/Next/Prev) -------------------------------
    def now(self, it: float) -> bool:
        if self.every_iter:
            it -= self.start_iter
            return math.floor(it / self.every_iter) > math.floor((it - 1) / self.every_iter)
        return False

    def next(self, it: float) -> int:
        if self.every_iter:
            it -= self.start_iter
            k = math.floor(it / self.every_iter)
            return int(-math.floor(-(k + 1) * self.every_iter) - it)
        return -1

    def prev(self, it: float) -> int:
        if self.every_iter:
            it -= self.start_iter
            k = math.floor((it - 1) / self.every_iter)
            return int(it + math.floor(-k * self.every_iter))
        return -1

    # -- design parameters (reference PAR_GET/SET/GRAD) --------------------------------
    def number_of_parameters(self) -> int:
        return 0

    def parameters(self, kind: int, data) -> int:
        return 0


class Action(Handler):
    kind = HANDLER_ACTION

    def init(self) -> int:
        it = self.node.get("Iterations")
        self.start_iter = self.solver.iter
        self.every_iter = self.solver.units.alt(it) if it is not None else 0.0
        if self.node.get("output") is not None:
            self.solver.set_output(self.node.get("output"))
        return 0


class Callback(Handler):
    kind = HANDLER_CALLBACK

    def init(self) -> int:
        it = self.node.get("Iterations")
        self.start_iter = self.solver.iter
        self.every_iter = self.solver.units.alt(it) if it is not None else 0.0
        return 0


class Design(Handler):
    kind = HANDLER_DESIGN


class GenericAction(Action):
    """Action executing its children (reference GenericAction)."""

    def init(self) -> int:
        self.stack = 0
        return super().init()

    def execute_internal(self) -> int:
        self.stack = 0
        for child in list(self.node):
            if not isinstance(child.tag, str):
                continue
            h = make_handler(child, self.solver)
            if h is None:
                if self.solver.permissive and child.tag not in REGISTRY:
                    continue
                raise HandlerError(f"Something wrong in {self.node.tag} (child {child.tag})")
            if h.kind & HANDLER_DESIGN:
                self.solver.hands.append(h)
                self.stack += 1
            elif h.kind & HANDLER_CALLBACK:
                if h.every_iter != 0:
                    self.solver.hands.append(h)
                    self.stack += 1
                else:
                    if h.do_it() not in (0, ITERATION_STOP, None):
                        raise HandlerError(f"Handler call error: {child.tag}")
        return 0

    def unstack(self):
        while self.stack > 0:
            h = self.solver.hands.pop()
            h.finish()
            self.stack -= 1

    def finish(self) -> int:
        if getattr(self, "stack", 0) > 0:
            self.unstack()
        return 0

    def solve_loop(self, action: Optional[str] = None) -> int:
        """the main time loop (reference acSolve::Init, src/Handlers/acSolve.cpp:5-47)"""
        s = self.solver
        from ..solver import ITER_LASTGLOB
        while True:
            my_next = self.next(s.iter)
            next_it = my_next
            for h in s.hands:
                it = h.next(s.iter)
                if 0 < it < next_it:
                    next_it = it
            if next_it <= 0:
                next_it = 1
            s.steps = next_it
            saved = s.iter_type
            if s.steps == my_next:
                s.iter_type |= ITER_LASTGLOB
            s.iterate(s.steps, action=action)
            s.iter_type = saved
            stop = False
            for h in list(s.hands):
                if h.now(s.iter):
                    r = h.do_it()
                    if r == ITERATION_STOP:
                        stop = True
                    elif r not in (0, None):
                        raise HandlerError(f"handler {h.node.tag} failed")
            if stop or self.now(s.iter):
                break
        return 0


class GenericContainer(GenericAction):
    def init(self) -> int:
        super().init()
        return self.execute_internal()

    def finish(self) -> int:
        self.unstack()
        return 0


def make_handler(node: ET.Element, solver) -> Optional[Handler]:
    """Factory: create the handler of an XML element and run its init()."""
    cls = REGISTRY.get(node.tag)
    if cls is None:
        if solver.permissive:
            log.warning(f"Unknown element {node.tag} (permissive: ignored)")
            return None
        raise HandlerError(f"Unknown XML element: {node.tag}")
    if not hasattr(solver, "_xml_parents"):
        solver._xml_parents = {c: p for p in solver.config_tree.iter() for c in p}
    h = cls(node, solver)
    r = h.init()
    if r not in (0, None):
        raise HandlerError(f"init of {node.tag} failed ({r})")
    return h
