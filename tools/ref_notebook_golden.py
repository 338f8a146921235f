#!/usr/bin/env python3
"""Extract the printed outputs of the reference's own T-scan notebook into a
test fixture (data only; the notebook is read as JSON text, nothing in it is
executed).

Source: /root/reference/scripts/plot_stiffness.ipynb, the stored outputs of a
real run of the Julia reference:
  cell 1   model of the data set: L = 24, J = 0.8, W = 1.0, n_imp = 0.0,
           μ = -1.4 (directory T_scan_L24_J0.8_W1.0_imp0.0_mu_-1.4, produced by
           scripts/batch_scan_T.jl:10-73 and summarised by
           scripts/batch_csv_summary_T.jl:23-166)
  cell 3   log-log fit of Delta_LocalPair / Delta_Loc over T > 10
  cell 5   log-log fit of Delta_Loc over T > 10
  cell 7   Beta column, rows 3..22
  cell 8   R = 1 / DC_Conductivity_mean, rows 3..22
  cell 11  1 / Beta (the T column), rows 0..22
Writes tests/golden/ref_Tscan_L24.json.
"""
from __future__ import annotations

import json
import os
import re
import sys

NB = "/root/reference/scripts/plot_stiffness.ipynb"
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "ref_Tscan_L24.json")


def cell_text(nb, i):
    out = []
    for o in nb["cells"][i].get("outputs", []):
        if "text" in o:
            out.append("".join(o["text"]))
        for k, v in o.get("data", {}).items():
            if k == "text/plain":
                out.append("".join(v))
    return "\n".join(out)


def series(text):
    """pandas Series repr -> {row index: value}"""
    vals = {}
    for line in text.splitlines():
        m = re.match(r"^\s*(\d+)\s+([-+0-9.eEinf]+)\s*$", line)
        if m:
            v = float(m.group(2))
            vals[int(m.group(1))] = v if v != float("inf") else None   # JSON null: printed as inf
    return vals


def fit(text):
    s = re.search(r"slope = ([-0-9.]+)", text)
    c = re.search(r"intercept = ([-0-9.]+)", text)
    return {"slope": float(s.group(1)), "intercept": float(c.group(1))}


def source(nb, i):
    return "".join(nb["cells"][i]["source"])


def main(nb_path=NB, out=OUT):
    with open(nb_path) as f:
        nb = json.load(f)
    src1 = source(nb, 1)
    model = {k: float(re.search(rf"^{k}\s*=\s*([-0-9.]+)", src1, re.M).group(1)) for k in ("L", "J", "W", "n_imp", "mu")}
    assert "T > 10" in source(nb, 3).replace("'T'] > 10", "T > 10") or "> 10" in source(nb, 3)
    T = series(cell_text(nb, 11))
    beta = series(cell_text(nb, 7))
    R = series(cell_text(nb, 8))
    rec = {
        "source": "scripts/plot_stiffness.ipynb stored outputs (cells 1, 3, 5, 7, 8, 11) of the reference's "
                  "T scan; produced by scripts/batch_scan_T.jl, reduced by scripts/batch_csv_summary_T.jl",
        "model": {"L": int(model["L"]), "J": model["J"], "W": model["W"], "n_imp": model["n_imp"],
                  "mu": model["mu"]},
        "T_rows": {str(k): v for k, v in sorted(T.items())},
        "beta_rows": {str(k): v for k, v in sorted(beta.items())},
        "R_rows": {str(k): v for k, v in sorted(R.items())},
        "fit_Delta_Loc_T_gt_10": fit(cell_text(nb, 5)),
        "fit_LocalPair_over_Loc_T_gt_10": fit(cell_text(nb, 3)),
        "display_digits": 7,
        "notes": "T_rows are 1/Beta as pandas printed them (the summary's T column is the run directory's "
                 "T rounded to 3 significant digits, batch_scan_T.jl:64, batch_csv_summary_T.jl:100-104); "
                 "R_rows = 1/mean(DC_Conductivity) over transport.csv (%.6f values), 7 significant digits.",
    }
    with open(out, "w") as f:
        json.dump(rec, f, indent=1)
    return rec


if __name__ == "__main__":
    r = main(*sys.argv[1:])
    print(json.dumps(r, indent=1))
