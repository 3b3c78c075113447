"""Phase timing of k_bil_dec (the RESCAL decoder's per-example kernel) from in-kernel
s_memrealtime stamps (100 MHz), on a bilinear BASELINE config (default C5).  Uses the
diagnostic library of tools/phase_stamps.py (-DRAE_STAMPS).  Diagnostic only.

    python tools/bil_stamps.py [--config c5] [--iters 10]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import phase_stamps as PS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c5")
    ap.add_argument("--iters", type=int, default=10)
    args = ap.parse_args()
    PS.build_diag()
    os.environ["RAE_LIB"] = PS.DIAG
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
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, 100, cfg["r"], cfg["m"],
                             cfg["s"], 0.0, 0.0, "adagrad", "stamps", cfg["dec"], False, True, False,
                             1.0, device=dev, graph_chunk=1, mfma_bf16=cfg.get("bf16", False))
    ind.compile_function()
    eng = ind.engine
    n1, n2 = ind.draw_epoch_negatives()
    eng.set_epoch_negatives(n1, n2)
    eng.run(0, 20, graph=False)
    torch.cuda.synchronize()
    grid = (C.c_int * 4)()
    lib.rae_debug_grid(eng.plan, grid)
    gf = list(grid)[0]
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    lib.rae_build_index(eng.plan, 20, args.iters, st)
    per = []
    vw = []
    nvw = ((cfg["r"] + 7) // 8) * ((cfg["r"] + 15) // 16)
    NSLOT = 8 if "RAE_MT_STAMP_PASS=1" in os.environ.get("RAE_VARIANT", "") else 6
    for it in range(args.iters):
        bf = torch.zeros(16384 + nvw * 8, dtype=torch.int64, device=dev)
        lib.rae_debug_stamps(eng.plan, C.c_void_p(bf.data_ptr()), 1)
        lib.rae_step_forward_at(eng.plan, 20 + it, st)
        lib.rae_debug_stamps(eng.plan, None, 1)
        lib.rae_step_update_at(eng.plan, 20 + it, st)
        torch.cuda.synchronize()
        allb = bf.cpu().numpy()
        v = allb[16384:16384 + nvw * 8].reshape(nvw, 8).astype(np.float64)[:, :NSLOT] / 100.0
        vw.append(np.concatenate([v[:, :1] - v[:, 0].min(), np.diff(v, axis=1)], axis=1))
        f = allb[:gf * 16].reshape(gf, 16).astype(np.float64)[:, :7] / 100.0   # -> us
        t0 = f[:, 0].min()
        per.append(np.concatenate([f[:, :1] - t0, np.diff(f, axis=1), f[:, -1:] - t0], axis=1))
    per = np.concatenate(per)
    cols = ["start", "ids+rec", "v,w+negrows", "dots", "coef+xy", "-", "record", "end"]
    print(f"k_bil_dec ({args.config}, {gf} workgroups), median/max us per phase:")
    print("  " + "  ".join(f"{c} {np.median(per[:, i]):.2f}/{per[:, i].max():.2f}"
                           for i, c in enumerate(cols)))
    st = np.array([v[:, 0] for v in vw])          # per iteration: WG start offsets
    print("k_bil_mt WG start offsets per iteration, p50/p90/p99/max us: " +
          "  ".join(f"{np.percentile(x, 50):.2f}/{np.percentile(x, 90):.2f}/{np.percentile(x, 99):.2f}/{x.max():.2f}"
                    for x in st))
    late = np.concatenate([np.nonzero(x > 5.0)[0] for x in st])
    if len(late):
        print(f"  late WGs (> 5 us) by blockIdx: {sorted(set(late.tolist()))[:40]} ... (XCD = blockIdx % 8: "
              f"{np.bincount(late % 8, minlength=8).tolist()})")
    vw = np.concatenate(vw)
    vcols = ["start", "staging", "operand loads", "barrier", "MFMA+contraction", "write", "dP",
             "dP stores"][:NSLOT]
    print(f"k_bil_mt pass {1 if NSLOT == 8 else 0} ({nvw} workgroups, wave 0 of each), median/max us per phase:")
    print("  " + "  ".join(f"{c} {np.median(vw[:, i]):.2f}/{vw[:, i].max():.2f}"
                           for i, c in enumerate(vcols)))
    end = vw.sum(axis=1)                          # wave 0's last stamp after the first WG start
    print("  wave-0 end after the first start, p10/p50/p90/p99/max us: " +
          "/".join(f"{np.percentile(end, q):.2f}" for q in (10, 50, 90, 99)) + f"/{end.max():.2f}")


if __name__ == "__main__":
    main()
