"""Collects the max elementwise relative error of every GPU parity check (test infrastructure).

`record()` is called by tests/test_gpu_parity.py's rel_close; at session end conftest.py writes
the table to $MPGNN_PARITY_REPORT (JSON lines) when that variable is set, so a GPU run can
commit the measured errors under profiles/."""
import json
import os

_ROWS: list = []


def record(what: str, err: float, tol: float, **extra) -> None:
    row = {"check": what, "max_rel_err": err, "tol": tol}
    row.update(extra)
    _ROWS.append(row)


def dump() -> None:
    path = os.environ.get("MPGNN_PARITY_REPORT")
    if not path or not _ROWS:
        return
    with open(path, "w") as f:
        for r in _ROWS:
            f.write(json.dumps(r) + "\n")
