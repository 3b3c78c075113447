"""Per-phase timing of the step kernels from in-kernel s_memrealtime stamps (100 MHz).

Builds/loads the diagnostic library (librae_hip_diag.so, compiled with -DRAE_STAMPS; the
product library has no stamps) and runs a few eager steps of a BASELINE config, then
prints, for k_forward, the median/max duration of each phase per workgroup kind and the
dispatch skew, and for k_update the per-task-type durations.  Diagnostic only: stamps add
barriers' worth of serialisation, so read shares, not absolute kernel time.

    python tools/phase_stamps.py [--config c3] [--iters 10] [--batch-size 100]
                                 [--G 8 --dp-update replicated|partitioned]

With --G > 1 the plan is rank 0 of a G-rank data-parallel plan whose collectives are no-ops
(tools/probes/dp_update_model.py's NoPeers): the update then runs over the global batch G*l.
"""
import argparse
import ctypes as C
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "relation-autoencoder_amd")
DIAG = os.path.join(PKG, "rae", "librae_hip_diag.so")
VARIANT = os.environ.get("RAE_VARIANT", "")      # extra -D flags: a diagnostic A/B build
sys.path.insert(0, PKG)
sys.path.insert(0, ROOT)


def build_diag():
    global DIAG
    import __graft_entry__ as ge
    if VARIANT:
        tag = VARIANT.replace("-D", "").replace("=", "").replace(" ", "_")
        DIAG = os.path.join(PKG, "rae", f"librae_hip_diag_{tag}.so")
    src = os.path.join(PKG, "csrc", "rae.hip")
    _lib = ge._lib_mod()
    if not os.path.exists(DIAG) or os.path.getmtime(DIAG) < max(os.path.getmtime(s) for s in _lib.source_files()):
        subprocess.run([ge.HIPCC, *_lib.BUILD_FLAGS, "-DRAE_STAMPS", "-DRAE_DIAG", *VARIANT.split(), src, "-o", DIAG],
                       check=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=100)
    ap.add_argument("--G", type=int, default=1)
    ap.add_argument("--dp-update", default="replicated")
    args = ap.parse_args()
    build_diag()
    os.environ["RAE_LIB"] = DIAG
    import torch
    import bench
    from rae import _lib
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    lib = _lib.load()
    lib.rae_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
    lib.rae_debug_grid.argtypes = [C.c_void_p, C.c_void_p]
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    dp = {}
    if args.G > 1:
        sys.path.insert(0, os.path.join(ROOT, "tools", "probes"))
        from dp_update_model import NoPeers
        dp = dict(world_size=args.G, rank=0, exchange=NoPeers(args.G), dp_update=args.dp_update)
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, args.batch_size,
                             cfg["r"], cfg["m"], cfg["s"], 0.0, 0.0, "adagrad", "stamps",
                             cfg["dec"], False, True, False, 1.0, device=dev, graph_chunk=1,
                             **dp)
    ind.compile_function()
    eng = ind.engine
    n1, n2 = ind.draw_epoch_negatives()
    eng.set_epoch_negatives(n1, n2)
    eng.run(0, 20, graph=False)
    torch.cuda.synchronize()
    grid = (C.c_int * 4)()
    lib.rae_debug_grid(eng.plan, grid)
    gf, gu, HA, HW = list(grid)
    HA = HW = 0
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    fw, up = [], []
    lib.rae_build_index(eng.plan, 20, args.iters, st)
    for it in range(args.iters):
        bf = torch.zeros(gf * 16, dtype=torch.int64, device=dev)
        bu = torch.zeros(gu * 4 * 4, dtype=torch.int64, device=dev)
        lib.rae_debug_stamps(eng.plan, C.c_void_p(bf.data_ptr()), 1)
        lib.rae_step_forward_at(eng.plan, 20 + it, st)
        torch.cuda.synchronize()
        lib.rae_debug_stamps(eng.plan, C.c_void_p(bu.data_ptr()), 0)
        lib.rae_step_update_at(eng.plan, 20 + it, st)
        torch.cuda.synchronize()
        fw.append(bf.cpu().numpy().reshape(gf, 16).astype(np.float64) / 100.0)   # -> us
        up.append(bu.cpu().numpy().reshape(gu * 4, 4).astype(np.float64))
    lib.rae_debug_stamps(eng.plan, None, 1)
    # the row-index kernel (built ahead of the steps, one launch per window of batches)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    lib.rae_build_index(eng.plan, 40, 64, st)
    e1.record()
    torch.cuda.synchronize()
    print(f"row-index build: {1e3 * e0.elapsed_time(e1) / 64:.2f} us per batch (64-batch launch)")

    print(f"config {args.config}: forward grid {gf} (A-index {HA}, W-index {HW}, examples "
          f"{gf - HA - HW}), update grid {gu}")
    kinds = {"A-index": slice(0, HA), "W-index": slice(HA, HA + HW), "example": slice(HA + HW, gf)}
    nph = {"A-index": 4, "W-index": 4, "example": 8}
    names = {"A-index": ["enumerate", "sort", "segment"], "W-index": ["enumerate", "sort", "segment"],
             "example": ["ids+C-cache", "encoder+gather", "C.P", "dots", "coef+dwC", "back+softmax",
                         "record"]}
    split = cfg["dec"] == "sp" and cfg["r"] * cfg["m"] > 32768
    if split:                                                    # split forward: k_sp_dec's stamps
        names["example"] = ["ids", "A-DMA+V", "dots", "coef", "weighted-rows", "record", "-"]
    spans = []
    for kind, sl in kinds.items():
        if sl.stop <= sl.start:
            continue
        per = []
        for f in fw:
            t0 = f[:, 0][f[:, 0] > 0].min()
            blk = f[sl, :nph[kind]]
            per.append(np.concatenate([blk[:, :1] - t0, np.diff(blk, axis=1), blk[:, -1:] - t0],
                                      axis=1))
            spans.append(f[:, :8].max() - t0)
        per = np.concatenate(per)
        cols = ["start"] + names[kind] + ["end"]
        print(f"  {kind:8s}: " + "  ".join(f"{c} {np.median(per[:, i]):.2f}/{per[:, i].max():.2f}"
                                           for i, c in enumerate(cols)))
    print(f"  forward span (first start -> last stamp): median {np.median(spans):.2f} us")
    sub = np.concatenate([f[HA + HW:gf] for f in fw])
    if np.all(sub[:, 8] > 0):
        print(f"  sub-phases: coef {np.median(sub[:, 8] - sub[:, 4]):.2f}  weighted-rows "
              f"{np.median(sub[:, 5] - sub[:, 8]):.2f}  C^T.dw {np.median(sub[:, 9] - sub[:, 5]):.2f}"
              f"  softmax-bwd {np.median(sub[:, 6] - sub[:, 9]):.2f}")
    if split and np.all(sub[:, 14] > 0):
        # k_sp_enc (slots 8-14): descriptor, feature ids, W rows + partial sums, S, softmax, record
        e = sub[:, 8:15]
        t0 = e[:, 0].min()
        print("  k_sp_enc: start {:.2f}/{:.2f}  desc {:.2f}  features {:.2f}  W-rows {:.2f}  S {:.2f}  "
              "softmax {:.2f}  record {:.2f}  end {:.2f}".format(
                  np.median(e[:, 0] - t0), np.max(e[:, 0] - t0),
                  *[np.median(e[:, q + 1] - e[:, q]) for q in range(6)], np.median(e[:, 6] - t0)))
    elif np.all(sub[:, 13] > 0) and np.all(sub[:, 12] > 0):
        print(f"  fast-path encoder: indices {np.median(sub[:, 10] - sub[:, 1]):.2f}  W-issue "
              f"{np.median(sub[:, 11] - sub[:, 10]):.2f}  W-wait+FMA(wave0) {np.median(sub[:, 12] - sub[:, 11]):.2f}"
              f"  barrier {np.median(sub[:, 13] - sub[:, 12]):.2f}  S+softmax {np.median(sub[:, 2] - sub[:, 13]):.2f}")
    elif np.all(sub[:, 11] > 0):
        print(f"  icache test: coef rep0 {np.median(sub[:, 10] - sub[:, 4]):.2f}  rep1 "
              f"{np.median(sub[:, 11] - sub[:, 10]):.2f}")
    clk = []
    for f in ([] if split else fw):
        ex = f[HA + HW:gf]
        clk += list((ex[:, 15] - ex[:, 14]) * 100.0 / ((ex[:, 7] - ex[:, 0]) * 100.0) * 100.0 / 100.0)
    if clk:
        print(f"  example-WG shader clock (s_memtime ticks / s_memrealtime): median {np.median(clk) * 100:.0f} MHz")
    tnames = ["C-tile", "R-tile", "Wb-tile", "cost", "A-row", "W-row", "A-heavy", "W-heavy",
              "A-vheavy", "W-vheavy"]
    allw = np.concatenate(up)
    valid = allw[:, 0] > 0
    allw = allw[valid]
    t0s = []
    for u in up:
        v = u[u[:, 0] > 0]
        t0s.append((v[:, 0].min(), v[:, 2].max(), v))
    print("  update (median/max us, first task of each wave):")
    for ty, nm in enumerate(tnames):
        d = []
        st_ = []
        en_ = []
        for t0, t1, v in t0s:
            sel = v[v[:, 1] == ty]
            d += list((sel[:, 2] - sel[:, 0]) / 100.0)
            st_ += list((sel[:, 0] - t0) / 100.0)
            en_ += list((sel[:, 2] - t0) / 100.0)
        if d:
            extra = ""
            if ty >= 4 and ty < 8:
                sg = np.concatenate([(v[v[:, 1] == ty][:, 3] - v[v[:, 1] == ty][:, 0]) / 100.0
                                     for _, _, v in t0s])
                extra = f"  (start->segment {np.median(sg):.2f}, segment->end {np.median(d) - np.median(sg):.2f})"
            print(f"    {nm:8s} n={len(d) // len(t0s):5d}  busy {np.median(d):.2f}/{np.max(d):.2f}"
                  f"  start {np.median(st_):.2f}/{np.max(st_):.2f}  end p50 {np.median(en_):.2f}"
                  f" p99 {np.percentile(en_, 99):.2f} max {np.max(en_):.2f}{extra}")
    mids = []
    for t0, t1, v in t0s:
        sel = v[(v[:, 1] == 0) & (v[:, 3] > 0)]
        mids += list(zip((sel[:, 3] - sel[:, 0]) / 100.0, (sel[:, 2] - sel[:, 3]) / 100.0))
    if mids:
        mids = np.array(mids)
        print(f"  icache test C-tile: start->rep1 {np.median(mids[:, 0]):.2f}  rep1->end {np.median(mids[:, 1]):.2f}")
    ends = np.concatenate([(v[:, 2] - t0) / 100.0 for t0, t1, v in t0s])
    starts = np.concatenate([(v[:, 0] - t0) / 100.0 for t0, t1, v in t0s])
    q = [10, 50, 90, 99, 100]
    print("  update waves (" + str(len(ends) // len(t0s)) + "): first-start pct " +
          " ".join(f"p{p} {np.percentile(starts, p):.2f}" for p in q) +
          " | last-end pct " + " ".join(f"p{p} {np.percentile(ends, p):.2f}" for p in q))
    print(f"  update span: median {np.median([(t1 - t0) / 100.0 for t0, t1, _ in t0s]):.2f} us")


if __name__ == "__main__":
    main()
