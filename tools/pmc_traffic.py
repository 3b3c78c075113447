"""HBM traffic per launch from two rocprofv3 PMC passes (FETCH_SIZE and WRITE_SIZE cannot
share a pass on gfx950: MI355X_MICROARCH.md "rocprofv3 PMC slots").

    python tools/pmc_traffic.py FETCH_DIR WRITE_DIR --config c3 [--out profiles/...json]

traffic = 2 x FETCH_SIZE + WRITE_SIZE  (gfx950 FETCH_SIZE tallies a wide coalesced read at
half its bytes -- MI355X_MICROARCH.md "HBM"), averaged over the launches of each kernel; the
step kernels are grouped as bench.py reports them, per STEP (a kernel launched twice a step,
k_bil_mt, counts twice; steps = launches of the update kernel): k_forward (SP: k_forward or the
split k_sp_* kernels; bilinear: the k_bil_* forward kernels) and k_update (k_vrec + k_update
[+ k_dense_w]; bilinear k_bil_update ...).  k_label (the labelling pass) is per launch.
FETCH_SIZE/WRITE_SIZE are in KB in rocprofv3's derived-counter output.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for fn in files:
        with open(fn) as fh:
            yield from csv.DictReader(fh)


def _group(name):
    n = name.split("(")[0].replace("void ", "").strip()
    base = n.split("<")[0]
    if base == "k_forward" or base in ("k_bil_enc", "k_bil_enc_fast", "k_bil_mt", "k_bil_dec", "k_bil_dp", "k_bil_dp2",
                                       "k_bil_fin", "k_sp_enc", "k_sp_cp", "k_sp_dec", "k_sp_ctdw",
                                       "k_sp_fin"):
        return "k_forward", base
    if base in ("k_update", "k_update_bil", "k_bil_update", "k_bil_prep", "k_bil_rows", "k_dense_w",
                "k_finalize_cost", "k_vrec"):
        return "k_update", base
    return None, base


def collect(d, counter):
    """per base kernel: (sum of counter over dispatches, dispatch count)"""
    tot = defaultdict(float)
    cnt = defaultdict(set)
    for row in _rows(d):
        if row.get("Counter_Name") != counter:
            continue
        name = row.get("Kernel_Name", "")
        _, base = _group(name)
        tot[base] += float(row["Counter_Value"])
        cnt[base].add(row.get("Dispatch_Id", row.get("Correlation_Id", len(cnt[base]))))
    return {k: (tot[k], len(cnt[k])) for k in tot}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default=None)
    args, extra = ap.parse_known_args()      # extra: the bench.py arguments of the passes
    fe = collect(args.fetch_dir, "FETCH_SIZE")
    wr = collect(args.write_dir, "WRITE_SIZE")
    per_kernel = {}
    for base in sorted(set(fe) | set(wr)):
        f, nf = fe.get(base, (0.0, 0))
        w, nw = wr.get(base, (0.0, 0))
        if not nf or not nw:
            continue
        per_kernel[base] = {"fetch_bytes": 1024.0 * f / nf, "write_bytes": 1024.0 * w / nw,
                            "launches": nf,
                            "traffic_bytes": 2.0 * 1024.0 * f / nf + 1024.0 * w / nw}
    out = {"source": f"rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE passes of bench.py "
                     f"--config {args.config} {' '.join(extra)}; traffic = 2*FETCH_SIZE + WRITE_SIZE per launch",
           "per_kernel": per_kernel}
    # per step: every kernel's total over the passes / the number of steps (the update kernel's
    # launches; one per step)
    steps = max((per_kernel[k]["launches"] for k in ("k_update", "k_update_bil", "k_bil_update")
                 if k in per_kernel), default=0)
    groups = defaultdict(float)
    for base, v in per_kernel.items():
        g, _ = _group(base)
        if g and steps:
            groups[g] += v["traffic_bytes"] * v["launches"] / steps
    out.update(groups)
    out["steps"] = steps
    # the library the passes profiled (bench.py compares it with the one it runs)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                    "relation-autoencoder_amd"))
    from rae import _lib
    out["build_id"] = _lib.library_build_id()
    txt = json.dumps(out, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as fh:
            fh.write(txt + "\n")


if __name__ == "__main__":
    main()
