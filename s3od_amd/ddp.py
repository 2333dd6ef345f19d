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
import time

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
        nbytes = flat_slice.numel() * flat_slice.element_size()
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
                    # ProcessGroupNCCL runs the collective on its own internal stream: wait() makes the comm
                    # stream wait for the collective's end event, so e0 -> e1 spans the RCCL kernel itself
                    # (e0 fires once the bucket is ready AND the previous bucket's collective has ended)
                    w.wait()
                    e1.record(self.stream)
                    self._ev.append((len(self._join), name, nbytes, e0, e1))
        else:
            t0 = time.perf_counter()
            w = dist.all_reduce(flat_slice, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            if self.timing:
                self._ev.append((len(self._join), name, nbytes, t0, w))
        self.works.append((w, flat_slice))

    def finish(self):
        timed = self.timing and bool(self.works)
        cuda = self.stream is not None
        if timed:
            if cuda:
                eb = torch.cuda.Event(enable_timing=True)
                eb.record()
            else:
                eb = time.perf_counter()
        done = {}
        for w, t in self.works:
            w.wait()
            if not cuda:
                done[id(w)] = time.perf_counter()      # host clock: issue -> wait() return (gloo, CPU tensors)
            if self.backend != "nccl":
                t.div_(self.world)
        if cuda:
            torch.cuda.current_stream().wait_stream(self.stream)
        if timed:
            if cuda:
                ej = torch.cuda.Event(enable_timing=True)
                ej.record()
            else:
                ej = time.perf_counter()
                self._ev = [(s, n, b, t0, done.get(id(w), ej) if not isinstance(w, float) else w)
                            for s, n, b, t0, w in self._ev]
            self._join.append((eb, ej))
        self.works.clear()

    def reset_timing(self, on=True):
        self.timing, self._ev, self._join = on, [], []

    @staticmethod
    def _union_ms(iv):
        """Length of the union of [start, end) intervals (ms)."""
        tot, cur_s, cur_e = 0.0, None, None
        for s, e in sorted(iv):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot

    def timing_report(self):
        """Communication report of the timed steps (synchronises).

        * ``buckets[].ms``: per bucket, the mean time from the bucket's all-reduce starting on the comm stream (bucket
          ready and the previous collective done) to the collective's end (CUDA: HIP events, the end one recorded on
          the comm stream behind ``Work.wait()``; gloo/CPU: host clock, issue -> ``wait()`` return);
        * ``allreduce_ms_per_step``: the union of the step's bucket intervals (time the link is busy), mean over steps;
        * ``bus_GBps``: 2 (N - 1) / N x bytes / that union;
        * ``comm_exposed_ms`` (+ ``_max``): the compute stream's wait from the end of the backward to the join in
          ``finish()`` -- the communication the backward did not hide."""
        if not self._join:
            return None
        cuda = self.stream is not None
        if cuda:
            torch.cuda.synchronize()
        steps = len(self._join)
        per, by_step = {}, {}
        origin = {}
        for s, name, nb, a, b in self._ev:
            if cuda:
                ref = origin.setdefault(s, a)    # the step's first bucket start (the comm stream runs buckets in order)
                t0, t1 = ref.elapsed_time(a), ref.elapsed_time(b)
            else:
                t0, t1 = a * 1e3, b * 1e3
            d = per.setdefault(name, {"bytes": nb, "ms": 0.0, "calls": 0})
            d["ms"] += t1 - t0
            d["calls"] += 1
            by_step.setdefault(s, []).append((t0, t1))
        if cuda:
            exposed = [eb.elapsed_time(ej) for eb, ej in self._join]
        else:
            exposed = [(ej - eb) * 1e3 for eb, ej in self._join]
        buckets = [{"bucket": k, "MB": round(v["bytes"] / 1e6, 2), "ms": round(v["ms"] / max(v["calls"], 1), 3)}
                   for k, v in per.items()]
        tot_b = sum(v["bytes"] for v in per.values())
        tot_ms = sum(self._union_ms(iv) for iv in by_step.values()) / steps
        return {"steps": steps, "buckets": buckets, "allreduce_ms_per_step": round(tot_ms, 3),
                "allreduce_MB_per_step": round(tot_b / 1e6, 2),
                "bus_GBps": round(tot_b / 1e6 / tot_ms * 2 * (self.world - 1) / self.world, 1) if tot_ms > 0 and self.world > 1 else None,
                "comm_exposed_ms": round(sum(exposed) / steps, 3), "comm_exposed_ms_max": round(max(exposed), 3),
                "clock": "HIP events" if cuda else "host perf_counter"}


def broadcast_parameters(model, src=0, group=None):
    """One-time broadcast of initial weights and BN buffers from rank 0."""
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src=src, group=group)
