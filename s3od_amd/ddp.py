"""Data-parallel gradient synchronisation (replaces Lightning's DDP/FSDP strategy,
synth_sod/.../train.py:116-125, config/backend/*.yaml).

One process per GPU (torchrun / torch.distributed.run), backend "nccl" = RCCL over xGMI.
The native backward calls ``on_ready(range, flat_slice)`` as soon as a block of parameter
gradients is final (seg_head first, then ViT layers 10..0, then the embeddings); each block is
all-reduced (mean) asynchronously on a dedicated HIP stream so communication overlaps the rest
of the backward.  ``finish()`` joins the outstanding collectives before the optimizer step.
``no_sync()`` skips the exchange for gradient-accumulation micro-batches (Lightning's
``accumulate_grad_batches``, backend/8gpu.yaml:6): the flat buffer keeps summing locally and the
last micro-batch's backward all-reduces the accumulated sum once.
Works with gloo on CPU tensors too (tests).
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist


class GradSync:
    def __init__(self, model=None, group=None):
        self.group = group
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.works = []
        self.stream = None
        self.enabled = True
        # S3OD_DDP_REHEARSE=1: issue the collectives even at world size 1 (exercises the RCCL
        # stream/event path on a one-GPU box; the mean over one rank is the identity)
        self.rehearse = os.environ.get("S3OD_DDP_REHEARSE", "0") == "1"
        # timing (bench.py sets it around its timed region): HIP events around every bucket's all-reduce on the
        # comm stream, and on the compute stream at backward end / after the join, so the exposed communication
        # of a step = the compute stream's wait for the last bucket
        self.timing = False
        self._ev = []          # (name, bytes, ev_start, ev_end) per bucket, comm stream
        self._join = []        # (ev_backward_end, ev_joined) per finish(), compute stream
        if model is not None:
            model.grad_ready_callback = self.on_ready
            model.grad_finish_callback = self.finish

    @contextlib.contextmanager
    def no_sync(self):
        prev, self.enabled = self.enabled, False
        try:
            yield
        finally:
            self.enabled = prev

    def on_ready(self, name, flat_slice):
        if not self.enabled or (self.world == 1 and not self.rehearse):
            return
        if flat_slice.is_cuda:
            if self.stream is None:
                self.stream = torch.cuda.Stream(device=flat_slice.device)
            ev = torch.cuda.Event()
            ev.record()
            with torch.cuda.stream(self.stream):
                self.stream.wait_event(ev)
                op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
                if self.timing:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(self.stream)
                w = dist.all_reduce(flat_slice, op=op, group=self.group, async_op=True)
                if self.timing:
                    e1.record(self.stream)
                    self._ev.append((name, flat_slice.numel() * flat_slice.element_size(), e0, e1))
        else:
            w = dist.all_reduce(flat_slice, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append((w, flat_slice))

    def finish(self):
        timed = self.timing and self.stream is not None and bool(self.works)
        if timed:
            eb = torch.cuda.Event(enable_timing=True)
            eb.record()
        for w, t in self.works:
            w.wait()
            if self.backend != "nccl":
                t.div_(self.world)
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
        if timed:
            ej = torch.cuda.Event(enable_timing=True)
            ej.record()
            self._join.append((eb, ej))
        self.works.clear()

    def reset_timing(self, on=True):
        self.timing, self._ev, self._join = on, [], []

    def timing_report(self):
        """Per-bucket all-reduce time on the comm stream and the exposed communication per step (the compute
        stream's wait from backward end to the join), averaged over the recorded steps (synchronises)."""
        if not self._join:
            return None
        torch.cuda.synchronize()
        steps = len(self._join)
        per = {}
        for name, nb, e0, e1 in self._ev:
            d = per.setdefault(name, {"bytes": nb, "ms": 0.0, "calls": 0})
            d["ms"] += e0.elapsed_time(e1)
            d["calls"] += 1
        exposed = [eb.elapsed_time(ej) for eb, ej in self._join]
        buckets = [{"bucket": k, "MB": round(v["bytes"] / 1e6, 2), "ms": round(v["ms"] / max(v["calls"], 1), 3)}
                   for k, v in per.items()]
        tot_b = sum(v["bytes"] for v in per.values())
        tot_ms = sum(v["ms"] for v in per.values()) / steps
        return {"steps": steps, "buckets": buckets, "allreduce_ms_per_step": round(tot_ms, 3),
                "allreduce_MB_per_step": round(tot_b / 1e6, 2),
                "bus_GBps": round(tot_b / 1e6 / tot_ms * 2 * (self.world - 1) / self.world, 1) if tot_ms > 0 and self.world > 1 else None,
                "comm_exposed_ms": round(sum(exposed) / steps, 3), "comm_exposed_ms_max": round(max(exposed), 3)}


def broadcast_parameters(model, src=0, group=None):
    """One-time broadcast of initial weights and BN buffers from rank 0."""
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src=src, group=group)
