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
                w = dist.all_reduce(flat_slice, op=op, group=self.group, async_op=True)
        else:
            w = dist.all_reduce(flat_slice, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.works.append((w, flat_slice))

    def finish(self):
        for w, t in self.works:
            w.wait()
            if self.backend != "nccl":
                t.div_(self.world)
        if self.stream is not None:
            torch.cuda.current_stream().wait_stream(self.stream)
        self.works.clear()


def broadcast_parameters(model, src=0, group=None):
    """One-time broadcast of initial weights and BN buffers from rank 0."""
    for t in list(model.parameters()) + list(model.buffers()):
        dist.broadcast(t.data, src=src, group=group)
