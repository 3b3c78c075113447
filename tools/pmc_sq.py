"""Per-kernel averages of the SQ counters of one rocprofv3 --pmc pass (counter_collection.csv).

    python tools/pmc_sq.py PMC_DIR [--kernels k_forward,k_update] [--out file.json]

WAVE_CYCLES / WAIT_* / ACTIVE_INST_* count quad-cycles summed over the kernel's waves
(MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES); the
fractions of WAVE_CYCLES say where a wave's time goes: parked on s_waitcnt / barriers
(WAIT_ANY), issue-stalled (WAIT_INST_ANY) or issuing (ACTIVE_INST_*)."""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--kernels", default="k_forward,k_update")
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    want = args.kernels.split(",")
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for fn in glob.glob(os.path.join(args.pmc_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "")
                base = name.split("(")[0].replace("void ", "").split("<")[0].strip()
                if base not in want:
                    continue
                tot[base][row["Counter_Name"]] += float(row["Counter_Value"])
                disp[base].add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    out = {}
    for k, c in tot.items():
        n = max(len(disp[k]), 1)
        avg = {cn: v / n for cn, v in c.items()}
        wc = avg.get("SQ_WAVE_CYCLES", 0.0)
        if wc:
            avg["fractions_of_wave_cycles"] = {cn: round(v / wc, 4) for cn, v in avg.items()
                                               if cn.startswith("SQ_") and cn != "SQ_WAVE_CYCLES"}
        avg["launches"] = n
        out[k] = avg
    txt = json.dumps(out, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
