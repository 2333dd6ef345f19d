"""Data-parallel logic on CPU with gloo, world_size 2 (the reference's `backend=cpu` idea,
config/backend/cpu.yaml): bucketed async gradient all-reduce = mean over ranks, bucket ranges of
the flat gradient layout partition every grad-bearing parameter exactly once, and the one-time
parameter broadcast."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from s3od_amd.ddp import GradSync, broadcast_parameters

        class Fake(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.w = torch.nn.Parameter(torch.full((4,), float(rank + 7)))
                self.register_buffer("rm", torch.full((2,), float(rank)))

        m = Fake()
        broadcast_parameters(m)
        flat = torch.arange(12, dtype=torch.float32) * (rank + 1)
        sync = GradSync()
        # buckets arrive in backward order (seg_head first, then layers high -> low)
        sync.on_ready("seg_head", flat[8:])
        sync.on_ready("layer1", flat[4:8])
        sync.on_ready("embeddings", flat[:4])
        sync.finish()
        q.put((rank, flat.tolist(), m.w.tolist(), m.rm.tolist()))
    finally:
        dist.destroy_process_group()


def test_gradsync_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    expect = [i * 1.5 for i in range(12)]          # mean of i*1 and i*2
    for rank, flat, w, rm in res:
        assert flat == pytest.approx(expect)
        assert w == [7.0] * 4 and rm == [0.0, 0.0]  # rank 0's values broadcast


def test_bucket_ranges_partition_grad_params():
    from s3od_amd.model import DPTSegmentation
    m = DPTSegmentation(init_seed=None)
    layout, ranges, total = m.grad_layout()
    assert total == 107_825_862                      # grad-bearing params
    spans = sorted(ranges.values())
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a0, b0), (a1, b1) in zip(spans, spans[1:]):
        assert b0 == a1                             # contiguous, non-overlapping
    names = [n for n, *_ in layout]
    assert len(names) == len(set(names))
    unused = set(m.unused_parameter_names())
    assert not unused & set(names)
    assert set(names) | unused == {n for n, _ in m.named_parameters()}
