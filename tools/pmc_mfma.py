"""MFMA utilisation per kernel from one rocprofv3 PMC pass with SQ_VALU_MFMA_BUSY_CYCLES,
SQ_BUSY_CYCLES and GRBM_GUI_ACTIVE (MI355X_MICROARCH.md "rocprofv3 PMC slots": 2 SQ + 1
GRBM counters fit one pass).

    python tools/pmc_mfma.py DIR [--cus 256] [--out profiles/...json]

mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs x 4 SIMDs), the gfx94x
MfmaUtil formula rocprofv3 falls back to on gfx950 (ROCm 7.2 ships no gfx950 derived
counters); MFMA_BUSY counts cycles (32 per v_mfma_f32_32x32x16_bf16, 16 per 16x16x32).
"""
import argparse
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import _rows  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--cus", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--stats", default=None, help="rocprofv3 kernel_stats.csv of the same command: "
                    "mfma_util_span = MFMA_BUSY / (avg duration x clock x CUs x 4)")
    ap.add_argument("--mhz", type=float, default=2400.0)
    a = ap.parse_args()
    dur = {}
    if a.stats:
        import csv
        with open(a.stats) as fh:
            for row in csv.DictReader(fh):
                base = row["Name"].split("(")[0].replace("void ", "").strip()
                dur[base] = float(row["AverageNs"]) * 1e-9
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for row in _rows(a.dir):
        base = row.get("Kernel_Name", "").split("(")[0].replace("void ", "").strip()
        tot[base][row["Counter_Name"]] += float(row["Counter_Value"])
        disp[base].add(row.get("Dispatch_Id", row.get("Correlation_Id")))
    out = {}
    for base, c in sorted(tot.items()):
        n = len(disp[base])
        busy, gui = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0), c.get("GRBM_GUI_ACTIVE", 0.0)
        if not n or not gui:
            continue
        out[base] = {"launches": n, "mfma_busy_cycles": busy / n, "gui_active_cycles": gui / n,
                     "sq_busy_cycles": c.get("SQ_BUSY_CYCLES", 0.0) / n,
                     "mfma_util": busy / (gui * a.cus * 4)}
        if base in dur:
            out[base]["avg_duration_us"] = dur[base] * 1e6
            out[base]["mfma_util_span"] = busy / n / (dur[base] * a.mhz * 1e6 * a.cus * 4)
    txt = json.dumps({"source": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
                                "GRBM_GUI_ACTIVE; mfma_util = MFMA_BUSY / (GUI_ACTIVE * CUs * 4); mfma_util_span "
                                "= MFMA_BUSY / (kernel duration * clock * CUs * 4)",
                      "per_kernel": out}, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
