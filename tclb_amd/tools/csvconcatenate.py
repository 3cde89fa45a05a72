"""csvconcatenate: join CSV logs of consecutive runs (reference tools/csvconcatenate):
``csvconcatenate out.csv in1.csv in2.csv ...`` keeps the first header and the union of
columns (missing values left empty)."""
from __future__ import annotations

import csv
import sys


def concatenate(out: str, inputs) -> int:
    rows, head = [], []
    for p in inputs:
        with open(p, newline="") as f:
            r = list(csv.DictReader(f))
        for row in r:
            for k in row:
                if k not in head:
                    head.append(k)
        rows.extend(r)
    with open(out, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=head)
        w.writeheader()
        w.writerows(rows)
    return 0


def main(argv=None) -> int:
    argv = sys.argv[1:] if argv is None else argv
    if len(argv) < 2:
        print("usage: csvconcatenate out.csv in1.csv [in2.csv ...]")
        return 2
    return concatenate(argv[0], argv[1:])


if __name__ == "__main__":
    sys.exit(main())
