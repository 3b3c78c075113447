"""The device training step behind ``func['train']`` and ``func['label_<split>']``.

Owns the HBM-resident dataset arrays, the exchange and cost buffers, and the C-ABI plan
(include/rae.h).  Two ways to drive it:

* ``train_call(batch, neg1, neg2)`` -- exactly the reference's compiled function signature
  (learning/OieInduction.py:146-149,189): host negatives for one batch in, cost out.
* ``run(first_batch, count)`` -- many steps back to back on per-epoch negatives resident in
  HBM, captured into HIP graphs (torch.cuda.CUDAGraph) so a step costs two kernel launches
  and no host round trip; per-batch costs stay on the device until the epoch ends.

Data-parallel: each rank computes its l examples of every global batch of L = G*l
examples; ``exchange`` (dist.py) all-gathers the per-example records between the forward
and the update kernels, so every rank applies the identical update.
"""
from __future__ import annotations

import ctypes as C
import os
import socket

import numpy as np
import torch

from . import _lib
from .data import batch_nnz_stats


_hip = None


def _upload_graph(g, stream):
    """hipGraphUpload the instantiated graph now, so its first replay does not pay for
    putting the kernel packets on the device (a first replay is otherwise ~1-2 us per step
    slower at 20 steps).  Best effort: a runtime without it just uploads on first replay."""
    global _hip
    try:
        if _hip is None:
            _hip = C.CDLL("libamdhip64.so")
            _hip.hipGraphUpload.argtypes = [C.c_void_p, C.c_void_p]
            _hip.hipGraphUpload.restype = C.c_int
        ex = g.raw_cuda_graph_exec()
        if ex:
            _hip.hipGraphUpload(C.c_void_p(ex), C.c_void_p(stream.cuda_stream))
            stream.synchronize()
    except (OSError, AttributeError, RuntimeError):
        pass


def check_p2p_devices(identities, cross_device: bool):
    """The peer-to-peer exchange's device guard: ranks whose GPUs differ are
    refused unless cross_device -- the kernels' stores into a peer GPU's memory have run on
    ranks sharing one GPU only (rae_p2p.hpp "Visibility across GPUs")."""
    devs = sorted(set(identities))
    if len(devs) > 1 and not cross_device:
        raise ValueError(
            f"dp_xchg='p2p' across {len(devs)} GPUs: the peer-to-peer exchange is verified on "
            "ranks sharing one GPU only; pass p2p_cross_device=True to run it across GPUs (or "
            "use dp_xchg='collective', the default)")


class DeviceSplit:
    """One split's CSR + entity ids in HBM (int32; values kept only if not all 1.0)."""

    def __init__(self, split, device):
        x = split.xFeats
        self.N = int(x.shape[0])
        self.d = int(x.shape[1])
        self.indptr_np = np.asarray(x.indptr, dtype=np.int64)
        if self.indptr_np[-1] >= 2 ** 31:
            raise ValueError("nnz exceeds int32 CSR addressing")
        self.indptr = torch.as_tensor(self.indptr_np.astype(np.int32), device=device)
        self.indices = torch.as_tensor(np.asarray(x.indices, dtype=np.int32), device=device)
        vals = np.asarray(x.data, dtype=np.float32)
        self.values = None if (vals.size == 0 or np.all(vals == 1.0)) else \
            torch.as_tensor(vals, device=device)
        self.args1 = torch.as_tensor(split.args1, device=device)
        self.args2 = torch.as_tensor(split.args2, device=device)


class TrainEngine:
    def __init__(self, model, optimizer, train_split, *, learning_rate, lambda1=0.0,
                 lambda2=0.0, world_size=1, rank=0, exchange=None, graph_chunk=64,
                 index_window=0, device=None, mfma_bf16=False, kernel_forms=None,
                 graph_absolute=False, dp_update="replicated", index_overlap=True,
                 p2p_cross_device=False, p2p_timeout=5.0):
        self.lib = _lib.load()
        self.model = model
        self.device = device if device is not None else model.params[0].device
        self.world_size = int(world_size)
        self.rank = int(rank)
        self.exchange = exchange
        self.graph_chunk = int(graph_chunk)
        dec = model.decoder
        self.m, self.r, self.s, self.l = model.m, model.r, model.s, model.l
        self.L = self.l * self.world_size
        self.split = train_split if isinstance(train_split, DeviceSplit) else \
            DeviceSplit(train_split, self.device)
        self.N = self.split.N
        self.nb = self.N // self.L                                     # OieInduction.py:98
        mbn, mrn = batch_nnz_stats(self.split.indptr_np, self.L)
        named = model.named_params()
        acc = {}
        if optimizer.accumulator is not None:
            acc = dict(zip(model.param_names, optimizer.accumulator))
        cfg = _lib.RaeConfig()
        cfg.decoder = _lib.RAE_DEC[dec.model_type]
        cfg.optimizer = _lib.RAE_OPT[optimizer.name]
        cfg.n_examples = self.N
        cfg.n_features = self.split.d
        cfg.n_entities = model.n
        cfg.relations = self.m
        cfg.embed = self.r
        cfg.neg_samples = self.s
        cfg.batch_size = self.l
        cfg.world_size = self.world_size
        cfg.rank = self.rank
        cfg.learning_rate = float(learning_rate)
        cfg.alpha = float(model.alpha)
        cfg.lambda1 = float(lambda1)
        cfg.lambda2 = float(lambda2)
        cfg.ext_reg = 1 if model.extended_reg else 0
        cfg.max_batch_nnz = mbn
        cfg.max_row_nnz = mrn
        cfg.neg_mode = _lib.RAE_NEG_PER_EPOCH
        cfg.neg_stride = self.N
        cfg.index_window = int(index_window)
        cfg.mfma_bf16 = 1 if mfma_bf16 else 0
        # kernel forms (include/rae.h RAE_SPFWD_* ...): {"sp_forward": "split", ...}; the
        # plan picks for the shape when a form is not named
        self.kernel_forms = dict(kernel_forms or {})
        if dp_update not in _lib.KERNEL_FORMS["dp_update"]:
            raise ValueError(f"dp_update must be one of {sorted(_lib.KERNEL_FORMS['dp_update'])}")
        self.kernel_forms.setdefault("dp_update", dp_update)
        # partitioned update with peers: rows are pulled from their owners before each forward
        self._dp = self.kernel_forms["dp_update"] == "partitioned" and self.world_size > 1
        if self._dp and exchange is None:
            raise ValueError("the partitioned data-parallel update needs the ranks' Exchange")
        # peer-to-peer exchange (include/rae.h RAE_XCHG_P2P): the kernels store rows and
        # records straight into the peers' IPC-mapped buffers -- no collective inside a step
        xchg = self.kernel_forms.get("dp_xchg", "collective")
        self._p2p = xchg != "collective" and self.world_size > 1
        if xchg != "collective" and self.kernel_forms["dp_update"] != "partitioned":
            raise ValueError("the peer-to-peer exchange runs the partitioned update")
        # pipelined form (RAE_XCHG_P2P_PIPE): every step pushes the NEXT batch's rows, so a
        # step needs the row lists of its batch + 1 (run() builds one batch past each window)
        # and a run whose first batch the previous step did not push starts with
        # rae_p2p_prologue (_p2p_start)
        self._pipe = self._p2p and xchg == "p2p_pipe"
        self._p2p_next = None        # batch the last queued step pushed rows for (signal out)
        self._p2p_valid = False      # ... pushed from the current negatives' lists
        self._ipc_bases = {}         # handle bytes -> this process's mapping of a peer allocation
        # ranks on different GPUs: the kernels' xGMI stores into a peer's memory (rae_p2p.hpp
        # "Visibility across GPUs") have run on ranks sharing one GPU only -- opt-in
        self._p2p_cross_device = bool(p2p_cross_device)
        self._p2p_timeout = float(p2p_timeout)
        for key, val in self.kernel_forms.items():
            if key not in _lib.KERNEL_FORMS or val not in _lib.KERNEL_FORMS[key]:
                raise ValueError(f"unknown kernel form {key}={val!r}")
            setattr(cfg, key, _lib.KERNEL_FORMS[key][val])
        self.cfg = cfg
        self.rec_floats = int(self.lib.rae_exchange_record_floats(C.byref(cfg)))
        self.exchange_buf = torch.zeros(int(self.lib.rae_exchange_floats(C.byref(cfg))),
                                        dtype=torch.float32, device=self.device)
        self.costs = torch.zeros(max(self.nb, 1), dtype=torch.float32, device=self.device)
        # per-epoch negatives live in fixed buffers (captured graphs keep their pointers)
        self.neg1 = torch.zeros((self.s, self.N), dtype=torch.int32, device=self.device)
        self.neg2 = torch.zeros((self.s, self.N), dtype=torch.int32, device=self.device)
        self.call_neg = torch.zeros((2, self.s, self.L), dtype=torch.int32, device=self.device)
        R3 = named.get("R", named.get("C"))
        bufs = _lib.RaeBuffers()
        p = _lib.ptr
        bufs.W, bufs.Wb, bufs.A, bufs.Ab = p(named["W"]), p(named["Wb"]), p(named["A"]), p(named["Ab"])
        bufs.C1, bufs.C2, bufs.R3 = p(named.get("C1")), p(named.get("C2")), p(R3)
        bufs.acc_W, bufs.acc_Wb = p(acc.get("W")), p(acc.get("Wb"))
        bufs.acc_A, bufs.acc_Ab = p(acc.get("A")), p(acc.get("Ab"))
        bufs.acc_C1, bufs.acc_C2 = p(acc.get("C1")), p(acc.get("C2"))
        bufs.acc_R3 = p(acc.get("R", acc.get("C")))
        bufs.indptr, bufs.indices = p(self.split.indptr), p(self.split.indices)
        bufs.values = p(self.split.values)
        bufs.args1, bufs.args2 = p(self.split.args1), p(self.split.args2)
        bufs.neg1, bufs.neg2 = p(self.neg1), p(self.neg2)
        bufs.exchange, bufs.costs = p(self.exchange_buf), p(self.costs)
        self._bufs = bufs
        self._keep = (named, acc, R3)
        self._named, self._acc = named, acc
        # row-exchange buffers of the partitioned update (sized from the row lists: _dp_caps)
        self._dp_caps = None
        self._dp_send = self._dp_recv = None
        self._stale = set()          # partitioned: {"params", "acc"} not gathered since a run
        self._dp_cap_max = (self.l * (2 + 2 * self.s), max(int(mbn), 1))   # rae.hip LA / LW
        handle = C.c_void_p()
        _lib.check(self.lib.rae_plan_create(C.byref(cfg), C.byref(bufs), C.byref(handle)),
                   "rae_plan_create")
        self.plan = handle
        if self._p2p:
            self._p2p_setup()
        self.index_window = int(self.lib.rae_index_window(self.plan))
        # a batch's row index is hash-partitioned (rae_index.hpp RAE_IDX_PART records per
        # partition) and a partition can overflow its LDS sort (a Zipf-heavy row at a large global
        # batch): run() checks the device error word after building each window's index, before
        # any step of the window applies an update (one host sync per window)
        self._graphs = {}
        self._epoch_mode = None
        # graph_absolute: every captured step carries its absolute batch index in the launch
        # (rae_step_*_at: no dependent device-cursor load at kernel start), one graph per
        # graph_chunk-step chunk of the epoch; otherwise one graph per chunk size, replayed
        # along the epoch by the device cursor
        self.graph_absolute = bool(graph_absolute)
        # batch the device cursor holds after this engine's last cursor-driven run (None:
        # unknown); run() skips its rae_set_cursor launch when the cursor already points at
        # the requested batch (consecutive runs of an epoch).  The plan counts every cursor
        # move made through the ABI (rae_cursor_moves): a move by anyone but this engine --
        # a direct rae_set_cursor / rae_advance_cursor on its plan -- changes the count, and
        # run() then sets the cursor again (cursor_moved() forces the same).
        self._cursor_at = None
        self._moves_seen = self._moves()
        # index_overlap: run() builds the next window's row index on a lowest-priority side
        # stream while the current window's steps run (the index is parameter independent; a
        # batch's slot is batch % index_window, so windows of half the ring never touch the
        # slots the steps in flight read).  Otherwise each window is built on the step stream
        # right before its steps.
        self.index_overlap = bool(index_overlap) and self.index_window >= 2
        self._win = self.index_window // 2 if self.index_overlap else self.index_window
        # pipelined p2p: each window's index covers one batch more (the last step's next
        # batch), so the ring holds a window + 1 beside the next window's build
        self._look = 1 if self._pipe else 0
        if self._look:
            self._win = max(1, self._win - 1)
        self._idx_stream = None
        if self.index_overlap:
            lo, _ = torch.cuda.Stream.priority_range()
            self._idx_stream = torch.cuda.Stream(self.device, priority=lo)
            # the runtime sets a stream's hardware queue up at its first use: 0.2-5.6 ms of
            # host time measured (tools/probes/bench_host_trace.py) -- here, not inside a run
            self._idx_stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self._idx_stream):
                torch.zeros(1, device=self.device).add_(1)
            self._idx_stream.synchronize()
        self._ready = None           # (lo, hi, negatives version, side-stream event): _mark_built
        self._neg_version = 0

    # ------------------------------------------------------------------ peer-to-peer exchange
    def _ipc_export(self, ptr: int):
        h = (C.c_char * _lib.RAE_IPC_HANDLE_BYTES)()
        off = C.c_int64()
        _lib.check(self.lib.rae_ipc_export(C.c_void_p(ptr), h, C.byref(off)), "rae_ipc_export")
        return bytes(h), int(off.value)

    def _ipc_map(self, handle: bytes, offset: int) -> int:
        base = self._ipc_bases.get(handle)
        if base is None:
            b = C.c_void_p()
            _lib.check(self.lib.rae_ipc_open(C.c_char_p(handle), C.byref(b)), "rae_ipc_open")
            base = self._ipc_bases[handle] = int(b.value)
        return base + offset

    def _device_identity(self):
        try:
            return str(torch.cuda.get_device_properties(self.device).uuid)
        except (AttributeError, RuntimeError):
            return f"{socket.gethostname()}:{self.device.index}"

    def _p2p_setup(self):
        """Trade IPC handles of this rank's exchange buffer, W, A, Ab and signal counters with
        every peer (a collective over the ranks' process group, once) and hand the peers'
        mappings to the plan (rae_set_peer).  Tensors sharing one allocation map it once.
        Ranks on different GPUs are refused unless p2p_cross_device=True (the
        cross-GPU stores have not run on hardware)."""
        named = self._named
        sig = self.lib.rae_p2p_signals(self.plan)
        mine = {"ex": self._ipc_export(self.exchange_buf.data_ptr()),
                "W": self._ipc_export(named["W"].data_ptr()),
                "A": self._ipc_export(named["A"].data_ptr()),
                "Ab": self._ipc_export(named["Ab"].data_ptr()),
                "sig": self._ipc_export(int(sig)),
                "dev": self._device_identity()}
        everyone = self.exchange.all_gather_object(mine)
        check_p2p_devices([e["dev"] for e in everyone], self._p2p_cross_device)
        _lib.check(self.lib.rae_set_p2p_timeout(self.plan, C.c_double(self._p2p_timeout)),
                   "rae_set_p2p_timeout")
        for p, e in enumerate(everyone):
            if p == self.rank:
                continue
            ptr = {k: self._ipc_map(*e[k]) for k in ("ex", "W", "A", "Ab", "sig")}
            _lib.check(self.lib.rae_set_peer(self.plan, p, C.c_void_p(ptr["ex"]),
                                             C.c_void_p(ptr["W"]), C.c_void_p(ptr["A"]),
                                             C.c_void_p(ptr["Ab"]), C.c_void_p(ptr["sig"])),
                       "rae_set_peer")

    # ------------------------------------------------------------------ partitioned update
    def _dp_caps_check(self):
        """After a row-index build: the longest peer row list of the batches just built,
        agreed over the ranks; (re)size the all-to-all blocks when a list would not fit (a
        resize drops the captured graphs, which hold the old buffers)."""
        ma, mw = C.c_int32(), C.c_int32()
        _lib.check(self.lib.rae_dp_list_max(self.plan, C.byref(ma), C.byref(mw)), "rae_dp_list_max")
        need_a = self.exchange.max_int(ma.value)
        need_w = self.exchange.max_int(mw.value)
        ca, cw = self._dp_caps or (0, 0)
        if self._dp_caps is not None and need_a <= ca and need_w <= cw:
            return
        # headroom: the first window's longest list is already the tail of many batches, and
        # a longer one later only re-sizes (a one-off): every padded row travels every step
        ca = min(max(ca, int(need_a * 1.04) + 16), self._dp_cap_max[0])
        cw = min(max(cw, int(need_w * 1.04) + 16), self._dp_cap_max[1])
        if self._p2p:                # capacities only: rows go straight into the peers' replicas
            _lib.check(self.lib.rae_set_dp_buffers(self.plan, None, None, ca, cw),
                       "rae_set_dp_buffers")
        else:
            blk = int(self.lib.rae_dp_block_floats(C.byref(self.cfg), ca, cw))
            self._dp_send = torch.zeros(self.world_size * blk, dtype=torch.float32,
                                        device=self.device)
            self._dp_recv = torch.zeros_like(self._dp_send)
            _lib.check(self.lib.rae_set_dp_buffers(self.plan, C.c_void_p(self._dp_send.data_ptr()),
                                                   C.c_void_p(self._dp_recv.data_ptr()), ca, cw),
                       "rae_set_dp_buffers")
        self._dp_caps = (ca, cw)
        self._graphs.clear()

    def stale(self, accumulators: bool = True) -> bool:
        """Partitioned update: whether this rank's replica misses rows its peers own that
        changed since the last sync_replicas (parameters; with `accumulators`, their AdaGrad
        state too).  Always False for the replicated update."""
        if not self._dp:
            return False
        return "params" in self._stale or (accumulators and "acc" in self._stale)

    def sync_replicas(self, accumulators: bool = True):
        """Partitioned update: gather every A / Ab / W row (and AdaGrad accumulator) from its
        owner, so every rank holds the whole current model (labelling, checkpoints, tests).
        A COLLECTIVE when anything is stale: every rank must call it (ReconstructInducer.gather
        before a rank-0-only save).  No-op when nothing is stale, and for the replicated update
        (replicas are identical after every step)."""
        if not self.stale(accumulators):
            return
        torch.cuda.synchronize(self.device)
        ts = [self._named["W"], self._named["A"], self._named["Ab"]]
        self._stale.discard("params")
        if accumulators and self._acc:
            ts += [self._acc.get("W"), self._acc.get("A"), self._acc.get("Ab")]
            self._stale.discard("acc")
        self.exchange.sync_rows(ts)

    # ------------------------------------------------------------------ helpers
    def _stream(self):
        return C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    def close(self):
        if getattr(self, "plan", None):
            rd = getattr(self, "_ready", None)
            if rd is not None and rd[3] is not None:
                rd[3].synchronize()
            self._ready = None
            self._graphs.clear()
            self.lib.rae_plan_destroy(self.plan)
            self.plan = None
            for base in self._ipc_bases.values():
                self.lib.rae_ipc_close(C.c_void_p(base))
            self._ipc_bases = {}

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def kernel_forms_in_use(self):
        """The kernel forms the plan resolved for its shape (rae_plan_forms), named as
        _lib.KERNEL_FORMS names them -- so the dict can be fed back as
        TrainEngine(kernel_forms=...) / bench.py --kernel-form to pin the same run:
        sp_forward fused|split (SP), bil_dp strided|staged|mtile (bilinear), bil_prep
        auto|kernel (bf16 bilinear: the forward writes the R-gradient operands, or k_bil_prep
        does), dp_update replicated|partitioned, priv_rows on|off (rows one record of the
        batch references updated per example, or by the row tasks), dp_dense records|partials
        (data-parallel SP: dw1 / dw2 per example in the exchange, or each rank's reduced dense
        gradients), heavy_chunk off|on (rows with at least 256 records of the global batch
        summed as parallel 128-record chunks).  Keys of forms that do not apply to the plan are left out."""
        out = _lib.RaeConfig()
        _lib.check(self.lib.rae_plan_forms(self.plan, C.byref(out)), "rae_plan_forms")
        F = _lib.KERNEL_FORMS
        name = {key: {code: n for n, code in F[key].items()} for key in F}
        sp = self.cfg.decoder == 0
        res = {}
        if sp:
            res["sp_forward"] = name["sp_forward"][out.sp_forward]
        else:
            res["bil_dp"] = name["bil_dp"][out.bil_dp]
            if self.cfg.mfma_bf16:
                res["bil_prep"] = name["bil_prep"][out.bil_prep]
        res["dp_update"] = name["dp_update"][out.dp_update]
        res["priv_rows"] = name["priv_rows"][out.priv_rows]
        if sp and self.world_size > 1:
            res["dp_dense"] = name["dp_dense"][out.dp_dense]
        if self.world_size > 1:
            res["dp_xchg"] = name["dp_xchg"][out.dp_xchg]
        res["heavy_chunk"] = name["heavy_chunk"][out.heavy_chunk]
        return res

    def _moves(self):
        return int(self.lib.rae_cursor_moves(self.plan))

    def set_cursor(self, batch: int):
        """Point the device cursor at global batch `batch` (stream-ordered)."""
        _lib.check(self.lib.rae_set_cursor(self.plan, int(batch), self._stream()), "rae_set_cursor")
        self._cursor_at = int(batch)
        self._moves_seen = self._moves()

    def cursor_moved(self):
        """Tell the engine the device cursor was driven outside run() (direct rae_set_cursor /
        rae_step_* calls on its plan): the next run() sets it again."""
        self._cursor_at = None

    def check(self, stream=None):
        """Raise if the plan's device error word is set.  stream=None: a blocking read (waits
        for all the device's queued work); else a read ordered on that stream only."""
        if stream is None:
            _lib.check(self.lib.rae_check(self.plan), "rae_check")
        else:
            _lib.check(self.lib.rae_check_on(self.plan, C.c_void_p(stream.cuda_stream)),
                       "rae_check_on")

    # ------------------------------------------------------------------ func['train']
    def train_call(self, batch_index, neg1, neg2) -> float:
        """One ``func['train'](batch_index, neg1, neg2)`` call (OieInduction.py:146-149):
        neg1/neg2 are (s, l) int32 host arrays; returns the batch cost as a Python float."""
        if self.world_size != 1:
            raise RuntimeError("train_call is the single-rank func['train'] path")
        n1 = np.ascontiguousarray(neg1, dtype=np.int32)
        n2 = np.ascontiguousarray(neg2, dtype=np.int32)
        if n1.shape != (self.s, self.l) or n2.shape != (self.s, self.l):
            raise ValueError(f"neg arrays must be ({self.s}, {self.l}), got {n1.shape}, {n2.shape}")
        b = int(batch_index)
        if not 0 <= b < self.nb:
            raise IndexError(f"batch index {b} out of range [0, {self.nb})")
        self._new_negatives()            # its index slot is rebuilt with the call's negatives
        self.call_neg[0].copy_(torch.from_numpy(n1))
        self.call_neg[1].copy_(torch.from_numpy(n2))
        st = self._stream()
        _lib.check(self.lib.rae_train_step(self.plan, b, C.c_void_p(self.call_neg[0].data_ptr()),
                                           C.c_void_p(self.call_neg[1].data_ptr()), st),
                   "rae_train_step")
        self._epoch_mode = None
        cost = float(self.costs[b].item())
        self.check()
        return cost

    # ------------------------------------------------------------------ epoch path
    def set_epoch_negatives(self, neg1, neg2):
        """(s, N) negatives of one epoch (OieInduction.py:183-184), host or device."""
        self._new_negatives()
        self.neg1.copy_(torch.as_tensor(np.asarray(neg1, dtype=np.int32)) if not
                        torch.is_tensor(neg1) else neg1)
        self.neg2.copy_(torch.as_tensor(np.asarray(neg2, dtype=np.int32)) if not
                        torch.is_tensor(neg2) else neg2)
        self._ensure_epoch_mode()

    def sample_epoch_negatives(self, sampler, mode: str = "device", seed: int = 0,
                               epoch: int = 0):
        """Fill the (s, N) per-epoch negative buffers on the device.
        mode "device": the shared RandomState draws neg1's then neg2's uniforms exactly as
          the reference does (OieInduction.py:183-184), the CDF search runs in HBM
          (rae_neg_sample) -- bit-identical to the host sampler, ~50x faster;
        mode "philox": uniforms generated on the device (rae_neg_sample_philox, counter =
          (epoch, buffer, draw)) -- no host work at all, not the reference's stream."""
        count = self.N * self.s
        self._new_negatives()
        if getattr(self, "_cum_dev", None) is None:
            self._cum_dev = torch.as_tensor(np.asarray(sampler.cum, dtype=np.float64),
                                            device=self.device)
        cum = C.c_void_p(self._cum_dev.data_ptr())
        n = int(self._cum_dev.numel())
        st = self._stream()
        for which, buf in enumerate((self.neg1, self.neg2)):
            if mode == "philox":
                off = (2 * int(epoch) + which) * count
                _lib.check(self.lib.rae_neg_sample_philox(cum, n, int(seed), off, count,
                                                          C.c_void_p(buf.data_ptr()), st),
                           "rae_neg_sample_philox")
            else:
                u = torch.from_numpy(sampler.draw_uniforms(count))
                if getattr(self, "_u_dev", None) is None or self._u_dev.numel() != count:
                    self._u_dev = torch.empty(count, dtype=torch.float64, device=self.device)
                self._u_dev.copy_(u)
                _lib.check(self.lib.rae_neg_sample(cum, n, C.c_void_p(self._u_dev.data_ptr()), count,
                                                   C.c_void_p(buf.data_ptr()), st), "rae_neg_sample")
        self._ensure_epoch_mode()

    def _ensure_epoch_mode(self):
        if self._epoch_mode is not True:
            _lib.check(self.lib.rae_set_negatives(self.plan, C.c_void_p(self.neg1.data_ptr()),
                                                  C.c_void_p(self.neg2.data_ptr()),
                                                  _lib.RAE_NEG_PER_EPOCH, self.N),
                       "rae_set_negatives")
            self._epoch_mode = True

    def _steps_eager(self, count, st, first=None, advance=True):
        """count steps from the device cursor (which then advances past them unless
        advance=False: a run's last graph, whose successor sets the cursor anyway), or (first
        given) at absolute batches first, first+1, ... (the cursor is not touched: every
        cursor-driven run sets it first)."""
        for i in range(count):
            if self._dp and not self._p2p:   # pull the rows this step's examples read
                if first is None:
                    _lib.check(self.lib.rae_dp_pack(self.plan, i, st), "rae_dp_pack")
                else:
                    _lib.check(self.lib.rae_dp_pack_at(self.plan, first + i, st), "rae_dp_pack_at")
                self.exchange.rows(self._dp_send, self._dp_recv)
                if first is None:
                    _lib.check(self.lib.rae_dp_unpack(self.plan, i, st), "rae_dp_unpack")
                else:
                    _lib.check(self.lib.rae_dp_unpack_at(self.plan, first + i, st),
                               "rae_dp_unpack_at")
            if first is None:
                _lib.check(self.lib.rae_step_forward(self.plan, i, st), "rae_step_forward")
            else:
                _lib.check(self.lib.rae_step_forward_at(self.plan, first + i, st),
                           "rae_step_forward_at")
            if self.exchange is not None and not self._p2p:
                self.exchange(self.exchange_buf)
            if first is None:
                _lib.check(self.lib.rae_step_update(self.plan, i, st), "rae_step_update")
            else:
                _lib.check(self.lib.rae_step_update_at(self.plan, first + i, st),
                           "rae_step_update_at")
        if first is None and advance:
            _lib.check(self.lib.rae_advance_cursor(self.plan, count, st), "rae_advance_cursor")

    def _graph(self, count, first=None, advance=True):
        key = (count if advance else ("last", count)) if first is None else (int(first), count)
        g = self._graphs.get(key)
        if g is None:
            # the capture calls rae_advance_cursor once (recorded, not run): not a real move
            in_sync = self._moves_seen == self._moves()
            g = torch.cuda.CUDAGraph()
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.graph(g, stream=s):
                self._steps_eager(count, self._stream(), first, advance)
            torch.cuda.current_stream(self.device).wait_stream(s)
            _upload_graph(g, s)
            self._graphs[key] = g
            if in_sync:
                self._moves_seen = self._moves()
        return g

    def _chunks(self, first_batch: int, count: int):
        """(first batch, steps) of every graph run() replays for these batches."""
        out = []
        for b, n in self.windows(first_batch, count):
            full, rem = divmod(n, self.graph_chunk)
            out += [(b + k * self.graph_chunk, self.graph_chunk) for k in range(full)]
            if rem:
                out.append((b + full * self.graph_chunk, rem))
        return out

    def _cursor_replays(self, first_batch: int, count: int, last_advance: bool = True):
        """Per window of run(first_batch, count): [(steps, advance), ...] of its cursor-driven
        graph replays.  last_advance=False: the run's very last graph does not advance the cursor
        (one node less; for a run no cursor-driven run follows directly -- run() records where
        the cursor stays, and the next run sets it)."""
        wins = self.windows(first_batch, count)
        out = []
        for wi, (_, n) in enumerate(wins):
            full, rem = divmod(n, self.graph_chunk)
            reps = [(self.graph_chunk, True)] * full + ([(rem, True)] if rem else [])
            if not last_advance and wi == len(wins) - 1 and reps:
                reps[-1] = (reps[-1][0], False)
            out.append(reps)
        return out

    def capture(self, count: int | None = None):
        """Capture the HIP graph of ``count`` steps (default: graph_chunk) without running it."""
        self._ensure_epoch_mode()
        self._graph(int(count or self.graph_chunk))

    def windows(self, first_batch: int, count: int):
        """The index windows run() walks: [(first batch, batches), ...] (half the ring each
        with index_overlap)."""
        out, b, end = [], int(first_batch), int(first_batch) + int(count)
        while b < end:
            n = min(self._win, end - b)
            out.append((b, n))
            b += n
        return out

    def graph_sizes(self, first_batch: int, count: int):
        """Step counts of the graphs run() replays for these batches: graph_chunk-step
        graphs, plus one graph for each window's remainder (so no step runs eagerly)."""
        if self.graph_chunk <= 1:
            return []
        sizes = []
        for _, n in self.windows(first_batch, count):
            full, rem = divmod(n, self.graph_chunk)
            sizes += [self.graph_chunk] * full + ([rem] if rem else [])
        return sizes

    def capture_for(self, first_batch: int, count: int, last_advance: bool = True):
        """Capture (without running) every graph run(first_batch, count, last_advance=...)
        will replay, so no capture lands inside a timed region."""
        self._ensure_epoch_mode()
        if self.graph_chunk <= 1:
            return
        if self.graph_absolute:
            for b, n in self._chunks(first_batch, count):
                self._graph(n, b)
            return
        for reps in self._cursor_replays(first_batch, count, last_advance):
            for n, adv in reps:
                self._graph(n, advance=adv)

    def build_index(self, first_batch: int, count: int):
        """Row index of batches [first_batch, first_batch+count) (one window at most)."""
        self._drain_prefetch()
        _lib.check(self.lib.rae_build_index(self.plan, int(first_batch), int(count), self._stream()),
                   "rae_build_index")
        self._mark_built(int(first_batch), int(first_batch) + int(count))
        if self._dp:
            self._dp_caps_check()

    def run(self, first_batch: int, count: int, graph: bool = True, index: bool = True,
            last_advance: bool = True, prefetch: bool | None = None, sync_peers: bool = True):
        """Run ``count`` consecutive global batches starting at ``first_batch`` on the epoch
        negatives; costs land in self.costs[first_batch:first_batch+count].  The row index
        of each window of batches is ready before the window's steps (index=False: the caller
        built it already, e.g. bench.py ahead of its timed region).  With index_overlap and
        prefetch (default: index), the index of the batches after each window -- the run's
        next window, or as many batches as the window after the run's last -- is built on the
        side stream, queued in front of the window's steps so it runs beside them.  With
        graph, every step runs inside a replayed HIP graph: graph_chunk-step graphs and one
        graph per window remainder (last_advance: see _cursor_replays).  sync_peers (the
        peer-to-peer exchange only): a host barrier of the ranks first -- a caller that has
        just met its peers (bench.py's timed region) may skip it."""
        self._ensure_epoch_mode()
        if self._dp:
            self._stale.update(("params", "acc"))
        if self._p2p and sync_peers:
            # a peer may have spent any time in host code since its last step (per-batch
            # evaluation, checkpoints): meet here so no wait kernel of this run starts its
            # bounded spin (rae_set_p2p_timeout) while a peer is still away
            self.exchange.barrier()
        pre = (index if prefetch is None else prefetch) and self.index_overlap
        replays = self._cursor_replays(first_batch, count, last_advance)
        wins = self.windows(first_batch, count)
        for wi, (b, n) in enumerate(wins):
            if index:
                self._index_ready(b, min(n + self._look, self.nb - b))
            if wi == 0 and self._pipe:
                self._p2p_start(b)
            nn_ = 0
            if pre:
                nn_ = wins[wi + 1][1] if wi + 1 < len(wins) else min(n, self.nb - (b + n))
            gate = None
            if nn_ > 0:
                # the next window's build may start once everything queued BEFORE this
                # window's steps is done (the previous window's steps read the slots it
                # writes); it is queued AFTER this window's replays, so its host calls never
                # stand between the GPU and the steps (66 vs 34 us of host queue
                # in front of a 20-step timed region)
                gate = torch.cuda.Event()
                gate.record(torch.cuda.current_stream(self.device))
            self._queue_window(b, n, wi, replays, graph)
            if gate is not None:
                self.prefetch_index(b + n, min(nn_ + self._look, self.nb - (b + n)), after=gate)
        if self._pipe and count > 0:
            # the run's last step pushed (and signalled) the rows of the batch after it
            self._p2p_next, self._p2p_valid = first_batch + count, True

    def _p2p_start(self, b: int):
        """Pipelined p2p: unless the previous step already pushed batch b's rows (from the
        current negatives' lists), push them now -- after consuming that step's signal for
        another batch (every rank runs the same batches, so every rank decides alike)."""
        if self._p2p_valid and self._p2p_next == b:
            return
        _lib.check(self.lib.rae_p2p_prologue(self.plan, int(b), 1 if self._p2p_next is not None else 0,
                                             self._stream()), "rae_p2p_prologue")

    def _queue_window(self, b, n, wi, replays, graph):
        """Queue the steps of window [b, b+n) (graph replays or eager launches)."""
        if graph and self.graph_chunk > 1 and self.graph_absolute:
            for cb, cn in self._chunks(b, n):
                self._graph(cn, cb).replay()
            return
        if self._cursor_at != b or self._moves_seen != self._moves():
            self.set_cursor(b)
        self._cursor_at = None              # until the window's launches are queued
        if not graph or self.graph_chunk <= 1:
            self._steps_eager(n, self._stream())
            self._cursor_at = b + n
        else:
            reps = replays[wi]
            for cnt, adv in reps:
                self._graph(cnt, advance=adv).replay()
            self._cursor_at = b + n - (0 if reps[-1][1] else reps[-1][0])
        self._moves_seen = self._moves()

    # ------------------------------------------------------------------ index overlap
    # self._ready = (lo, hi, negatives version, event): batches [lo, hi) have their row index
    # in the ring; event (or None) marks the end of a side-stream build not yet waited for.
    def _mark_built(self, x: int, y: int, event=None):
        lo, hi, ver, ev = self._ready if self._ready else (x, x, self._neg_version, None)
        if ver != self._neg_version or x != hi:      # not contiguous: a new range
            lo, ev = x, None
        self._ready = (max(lo, y - self.index_window), y, self._neg_version, event or ev)

    def _covered(self, b: int, e: int) -> bool:
        rd = self._ready
        return rd is not None and rd[2] == self._neg_version and rd[0] <= b and e <= rd[1]

    def prefetch_index(self, first_batch: int, count: int, after=None):
        """Start the row index of batches [first_batch, first_batch+count) -- the part not
        already built -- on the side stream, behind everything queued on the step stream so
        far (or, `after` given, behind that event of the step stream), in front of whatever is
        queued after.  Steps queued after the point it waits for may read batches
        >= first_batch + count - index_window only (a window of half the ring ahead of the
        window being run satisfies that)."""
        if not self.index_overlap:
            raise RuntimeError("prefetch_index needs index_overlap")
        x, y = int(first_batch), int(first_batch) + int(count)
        rd = self._ready
        if rd is not None and rd[2] == self._neg_version and rd[0] <= x <= rd[1]:
            x = max(x, rd[1])                        # extend the built range
        if y <= x:
            return
        if after is None:
            self._idx_stream.wait_stream(torch.cuda.current_stream(self.device))
        else:
            self._idx_stream.wait_event(after)
        _lib.check(self.lib.rae_build_index(self.plan, x, y - x,
                                            C.c_void_p(self._idx_stream.cuda_stream)),
                   "rae_build_index")
        done = torch.cuda.Event()
        done.record(self._idx_stream)
        self._mark_built(x, y, done)

    def _index_ready(self, b: int, n: int):
        """The window [b, b+n)'s index before its steps: already in the ring (a side-stream
        build the step stream then waits for), else built on the step stream; then the
        overflow check (host sync) and, partitioned, the row-list capacities.  The check of a
        side-stream build reads the error word on the side stream: the host waits for that
        build only, not for the steps still queued on the step stream (a blocking
        null-stream read there left a GPU bubble at every window boundary)."""
        if self._covered(b, b + n):
            ev = self._ready[3]
            if ev is not None:
                torch.cuda.current_stream(self.device).wait_event(ev)
                self._ready = self._ready[:3] + (None,)
                self.check(self._idx_stream)
            else:
                self.check()
        else:
            self._drain_prefetch()
            _lib.check(self.lib.rae_build_index(self.plan, b, n, self._stream()),
                       "rae_build_index")
            self._mark_built(b, b + n)
            self.check()
        if self._dp:
            self._dp_caps_check()

    def _drain_prefetch(self):
        """A side-stream build still in flight: the step stream waits for it (it uses the
        plan's index scratch and reads the negatives)."""
        if self._ready is not None and self._ready[3] is not None:
            torch.cuda.current_stream(self.device).wait_event(self._ready[3])
            self._ready = self._ready[:3] + (None,)

    def _new_negatives(self):
        self._drain_prefetch()
        self._neg_version += 1
        self._p2p_valid = False      # rows pushed from the old lists: push the next run's again

    # ------------------------------------------------------------------ labelling
    def label(self, split: DeviceSplit, row0: int, nrows: int, probs: bool = True):
        """labels (int64) and probs (fp32) of rows [row0, row0+nrows) of a split with the
        current W/Wb (RelationClassifier.py:39-48).  Partitioned update with stale rows: the
        W rows are gathered from their owners first -- a collective, so every rank labels (or
        ReconstructInducer.gather() ran on every rank before a single rank labels)."""
        if self.stale(accumulators=False):   # partitioned update: gather W from its owners
            self.sync_replicas(accumulators=False)
        lab = torch.empty(nrows, dtype=torch.int64, device=self.device)
        pr = torch.empty((nrows, self.m), dtype=torch.float32, device=self.device) if probs else None
        W, Wb = self.model.params[0], self.model.params[1]
        _lib.check(self.lib.rae_label(
            C.c_void_p(split.indptr.data_ptr()), C.c_void_p(split.indices.data_ptr()),
            C.c_void_p(split.values.data_ptr()) if split.values is not None else None,
            C.c_void_p(W.data_ptr()), C.c_void_p(Wb.data_ptr()), self.m, int(row0), int(nrows),
            C.c_void_p(lab.data_ptr()), C.c_void_p(pr.data_ptr()) if pr is not None else None,
            self._stream()), "rae_label")
        return lab, pr
