"""Levelled, rank-tagged logger (reference: myprint levels debug0..ERROR,
src/Global.h.Rt:87-165, src/Global.cpp.Rt:203-246).  Below NOTICE only rank 0 prints."""
from __future__ import annotations

import os
import sys
import time

LEVELS = {"debug2": 0, "debug1": 1, "debug0": 2, "output": 3, "notice": 4, "NOTICE": 5, "warning": 6,
          "WARNING": 7, "error": 8, "ERROR": 9}


class Logger:
    def __init__(self):
        self.level = int(os.environ.get("TCLB_VERBOSITY", "3"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.color = sys.stderr.isatty()
        self.t0 = time.time()

    def _p(self, lvl: int, msg: str):
        if lvl < self.level:
            return
        if lvl < 6 and self.rank != 0:
            return
        tag = {8: "error", 9: "ERROR", 6: "warning", 7: "WARNING"}.get(lvl, "")
        pre = f"[{self.rank}] " + (f"{tag}: " if tag else "")
        out = sys.stderr if lvl >= 6 else sys.stdout
        if self.color and lvl >= 6:
            out.write(f"\033[1;31m{pre}{msg}\033[0m\n")
        else:
            out.write(f"{pre}{msg}\n")
        out.flush()

    def debug(self, m): self._p(1, m)
    def output(self, m): self._p(3, m)
    def info(self, m): self._p(3, m)
    def notice(self, m): self._p(4, m)
    def NOTICE(self, m): self._p(5, m)
    def warning(self, m): self._p(6, m)
    def WARNING(self, m): self._p(7, m)
    def error(self, m): self._p(8, m)
    def ERROR(self, m): self._p(9, m)


log = Logger()
