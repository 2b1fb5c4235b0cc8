"""Collects the max elementwise relative error of every GPU parity check (test infrastructure).

`record()` is called by tests/test_gpu_parity.py's rel_close; at session end conftest.py writes
the table to $MPGNN_PARITY_REPORT (JSON lines) when that variable is set, so a GPU run can
commit the measured errors under profiles/."""
import json
import os

_ROWS: list = []


def record(what: str, err: float, tol: float, **extra) -> None:
    """One row per check: the pytest node id that made it (PYTEST_CURRENT_TEST: file::test[params]),
    the label, the errors and the bar; `bar_ratio` = how close the deciding error came to its bar
    (elementwise vs tol when that passes; else the float64-truth error vs factor x the fp32
    reference path's own error)."""
    node = os.environ.get("PYTEST_CURRENT_TEST", "").rsplit(" (", 1)[0]
    row = {"test": node, "check": what, "max_rel_err": err, "tol": tol}
    row.update(extra)
    if err <= tol or "e_gpu64" not in extra:
        row["bar_ratio"] = err / tol if tol > 0 else None
        row["decided_by"] = "elementwise vs fp32 reference"
    else:
        bar = max(tol, extra.get("cpu_factor", 2.0) * extra["e_cpu64"])
        row["bar_ratio"] = extra["e_gpu64"] / bar if bar > 0 else None
        row["decided_by"] = "float64 truth vs factor x fp32 reference error"
    _ROWS.append(row)


def dump() -> None:
    path = os.environ.get("MPGNN_PARITY_REPORT")
    if not path or not _ROWS:
        return
    with open(path, "w") as f:
        for r in _ROWS:
            f.write(json.dumps(r) + "\n")
