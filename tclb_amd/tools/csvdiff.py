"""csvdiff: compare two CSV files column by column (reference tools/csvdiff).

Numeric columns agree when max|a-b| / ((max|a| + max|b|)/2) <= limit (columns whose mean
magnitude is below the limit are skipped); other columns must be identical.  Columns
matching any of the comma-separated ``--discard`` regexps are ignored.
Exit status: 0 equal, 1 different shape, 2 different header, 3 values differ."""
from __future__ import annotations

import argparse
import csv
import re
import sys
from typing import Dict, List


def read(path: str) -> Dict[str, List[str]]:
    with open(path, newline="") as f:
        rows = list(csv.reader(f))
    if not rows:
        raise SystemExit(f"{path} is not a valid CSV file")
    head = [h.strip().strip('"') for h in rows[0]]
    cols: Dict[str, List[str]] = {h: [] for h in head}
    for r in rows[1:]:
        if not r:
            continue
        for h, v in zip(head, r):
            cols[h].append(v.strip())
    return cols


def _num(v: List[str]):
    try:
        return [float(x) for x in v]
    except ValueError:
        return None


def csvdiff(a: str, b: str, limit: float = 1e-10, discard: str = "") -> int:
    pats = [p for p in discard.split(",") if p]
    keep = lambda n: not any(re.search(p, n) for p in pats)   # noqa: E731
    t1 = {k: v for k, v in read(a).items() if keep(k)}
    t2 = {k: v for k, v in read(b).items() if keep(k)}
    n1 = (len(next(iter(t1.values()), [])), len(t1))
    n2 = (len(next(iter(t2.values()), [])), len(t2))
    if n1 != n2:
        print(f"dimensions not identical: {n1} {n2}")
        return 1
    if sorted(t1) != sorted(t2):
        print(f"names (header) not identical:\n{sorted(t1)}\n{sorted(t2)}")
        return 2
    eps = abs(limit)
    for name in t1:
        x, y = _num(t1[name]), _num(t2[name])
        if x is not None and y is not None:
            div = (max(map(abs, x), default=0) + max(map(abs, y), default=0)) / 2
            if div >= eps:
                d = max((abs(p - q) for p, q in zip(x, y)), default=0.0)
                if d / div > eps:
                    print(f"Differ at {name}\n  max(abs(a-b))     : {d}\n  max(abs(a-b)/div) : {d / div}\n  eps               : {eps}")
                    return 3
        elif t1[name] != t2[name]:
            print(f"Differ at {name}")
            return 3
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="compare two CSV files")
    ap.add_argument("-a", "--filea", required=True)
    ap.add_argument("-b", "--fileb", required=True)
    ap.add_argument("-x", "--limit", type=float, default=1e-10)
    ap.add_argument("-d", "--discard", default="")
    a = ap.parse_args(argv)
    return csvdiff(a.filea, a.fileb, a.limit, a.discard)


if __name__ == "__main__":
    sys.exit(main())
