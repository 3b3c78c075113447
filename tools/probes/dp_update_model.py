"""Single-GPU cost model of the data-parallel update at world size G (no peers: the
collectives are no-ops, the other ranks' records stay zero -- a timing probe only).

    python tools/probes/dp_update_model.py [--G 8] [--l 100] [--config c3]

Times, per step, rank 0's forward (l examples), the partitioned form's row pull kernels
(rae_dp_pack + rae_dp_unpack, without the all-to-all) and the update over the global batch
L = G*l -- replicated (every referenced row) vs partitioned (the rows rank 0 owns) -- with the
kernels' own dispatch timestamps (rae_time_next), plus the bytes each all-to-all / all-gather
would move.  DESIGN.md sec. 4 uses it for the per-step model of the 8-GPU run."""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "relation-autoencoder_amd"))
sys.path.insert(0, ROOT)


class NoPeers:
    def __init__(self, G):
        self.world_size, self.rank = G, 0

    def __call__(self, buf):
        pass

    def rows(self, send, recv):
        pass

    def max_int(self, v):
        return int(v)

    def sync_rows(self, ts):
        pass


def main():
    import torch
    import bench
    from rae.data import synthetic_dataset
    from rae.inducer import ReconstructInducer
    ap = argparse.ArgumentParser()
    ap.add_argument("--G", type=int, default=8)
    ap.add_argument("--l", type=int, default=100)
    ap.add_argument("--config", default="c3")
    ap.add_argument("--iters", type=int, default=50)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    data, gold = synthetic_dataset(cfg["N"], cfg["d"], cfg["ntrue"], seed=1234)
    res = {"G": args.G, "l": args.l, "config": args.config}
    for mode in ("replicated", "partitioned"):
        ind = ReconstructInducer(data, gold, np.random.RandomState(2), 1, 0.1, args.l, cfg["r"],
                                 cfg["m"], cfg["s"], 0.0, 0.0, "adagrad", "dpm", cfg["dec"], False,
                                 True, False, 1.0, device=dev, world_size=args.G, rank=0,
                                 exchange=NoPeers(args.G), graph_chunk=1,
                                 mfma_bf16=cfg.get("bf16", False), dp_update=mode)
        ind.compile_function()
        eng = ind.engine
        eng.sample_epoch_negatives(ind.negativeSampler, "device")
        n = min(args.iters, eng.nb, eng.index_window)
        eng.build_index(0, n)
        eng.set_cursor(0)
        lib, plan = eng.lib, eng.plan
        st = C.c_void_p(torch.cuda.current_stream().cuda_stream)

        def ev():
            h = C.c_void_p()
            assert lib.rae_event_create(C.byref(h)) == 0
            return h
        t = {"forward": [], "pack": [], "unpack": [], "update": []}
        evs = []
        for i in range(n):
            e = {k: (ev(), ev()) for k in t}
            if mode == "partitioned":
                assert lib.rae_time_next(plan, *e["pack"]) == 0
                assert lib.rae_dp_pack(plan, i, st) == 0, lib.rae_last_error()
                assert lib.rae_time_next(plan, *e["unpack"]) == 0
                assert lib.rae_dp_unpack(plan, i, st) == 0, lib.rae_last_error()
            assert lib.rae_time_next(plan, *e["forward"]) == 0
            assert lib.rae_step_forward(plan, i, st) == 0
            assert lib.rae_time_next(plan, *e["update"]) == 0
            assert lib.rae_step_update(plan, i, st) == 0
            evs.append(e)
        torch.cuda.synchronize()
        for e in evs:
            for k in t:
                if k in ("pack", "unpack") and mode != "partitioned":
                    continue
                v = C.c_float()
                if lib.rae_event_elapsed_ms(e[k][0], e[k][1], C.byref(v)) == 0:
                    t[k].append(v.value * 1e3)
        out = {k: float(np.median(v[3:])) for k, v in t.items() if v}
        rec = eng.rec_floats * 4
        out["records_allgather_in_bytes"] = (args.G - 1) * args.l * rec
        if mode == "partitioned":
            ca, cw = eng._dp_caps
            blk = int(lib.rae_dp_block_floats(C.byref(eng.cfg), ca, cw)) * 4
            out["rows_alltoall_in_bytes"] = (args.G - 1) * blk
            out["row_caps"] = [ca, cw]
        res[mode] = out
        ind._drop_engine()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
