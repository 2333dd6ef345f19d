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


def _worker_model(rank, world, port, q):
    """The model's real flat-gradient layout and bucket ranges, driven through _grad_ready_hook in
    the native backward's order (seg_head, layer10..layer0, embeddings) and _after_backward
    (-> GradSync.finish); then a no_sync() accumulation micro-batch followed by a synced one."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from s3od_amd.model import DPTSegmentation
        from s3od_amd.ddp import GradSync
        m = DPTSegmentation(init_seed=None)
        sync = GradSync(m)
        G = m._grad_views()
        buf = G["_flat"]
        n = buf.numel()
        base = torch.arange(n, dtype=torch.float32) % 997

        def backward_hooks():
            m._grad_ready_hook("seg_head")
            for i in reversed(range(11)):
                m._grad_ready_hook(f"layer{i}")
            m._grad_ready_hook("embeddings")
            m._after_backward()

        buf.copy_(base * (rank + 1))
        backward_hooks()
        ok1 = bool(torch.equal(buf, base * 1.5))            # mean of x1 and x2
        # accumulation: micro-batch 1 under no_sync (local only), micro-batch 2 synced
        buf.zero_()
        with sync.no_sync():
            buf.add_(base * (rank + 1))
            backward_hooks()
        local_ok = bool(torch.equal(buf, base * (rank + 1)))  # untouched by the exchange
        buf.add_(base * (rank + 1))
        backward_hooks()
        ok2 = bool(torch.equal(buf, base * 3.0))             # mean over ranks of 2x(rank+1)
        # every parameter's .grad is a view of the exchanged buffer
        p = dict(m.named_parameters())["encoder.model.layer.3.mlp.up_proj.weight"]
        ok3 = p.grad.data_ptr() >= buf.data_ptr() and bool(p.grad.abs().sum() > 0)
        q.put((rank, ok1, local_ok, ok2, ok3, n))
    finally:
        dist.destroy_process_group()


def test_gradsync_model_layout_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_model, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, ok1, local_ok, ok2, ok3, n in res:
        assert n == 107_825_862
        assert ok1 and local_ok and ok2 and ok3, (rank, ok1, local_ok, ok2, ok3)


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


def _worker_nan(rank, world, port, q):
    """Only rank 1 counted a non-finite loss: both ranks must raise at the same check."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from s3od_amd.train import nan_guard
        clean = torch.zeros((), dtype=torch.int32)
        nan_guard(clean, world, "step 0")                     # nobody saw a NaN: no raise anywhere
        bad = torch.tensor(1 if rank == 1 else 0, dtype=torch.int32)
        try:
            nan_guard(bad, world, "step 1")
            raised = False
        except FloatingPointError:
            raised = True
        dist.barrier()                                        # both ranks are still in lock-step
        q.put((rank, raised))
    finally:
        dist.destroy_process_group()


def test_nan_guard_all_ranks_raise_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_nan, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: True, 1: True}


def _worker_timing(rank, world, port, q):
    """GradSync's communication report at world 2 (gloo, CPU): the keys bench.py's `comm` object carries, per-bucket
    intervals that end after they start, and the per-step link-busy time as the UNION of the bucket intervals (never
    more than their sum)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from s3od_amd.ddp import GradSync
        sync = GradSync()
        sync.reset_timing(True)
        flat = torch.ones(3 << 20, dtype=torch.float32) * (rank + 1)
        for _ in range(2):                                   # two "steps"
            sync.on_ready("seg_head", flat[2 << 20:])
            sync.on_ready("layer0", flat[1 << 20:2 << 20])
            sync.on_ready("embeddings", flat[:1 << 20])
            sync.finish()
        rep = sync.timing_report()
        sync.reset_timing(False)
        q.put((rank, rep, float(flat[0])))
    finally:
        dist.destroy_process_group()


def test_gradsync_timing_report_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_timing, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    for rank, rep, v0 in res:
        assert v0 == pytest.approx(1.5)                      # mean of 1 and 2, then the mean of 1.5 and 1.5
        assert rep is not None and rep["steps"] == 2
        for k in ("buckets", "allreduce_ms_per_step", "allreduce_MB_per_step", "bus_GBps", "comm_exposed_ms",
                  "comm_exposed_ms_max", "clock"):
            assert k in rep, k
        assert [b["bucket"] for b in rep["buckets"]] == ["seg_head", "layer0", "embeddings"]
        assert all(b["ms"] >= 0 for b in rep["buckets"])
        assert rep["allreduce_MB_per_step"] == pytest.approx(3 * 4 * (1 << 20) / 1e6, rel=1e-3)
        assert 0 < rep["allreduce_ms_per_step"] <= sum(b["ms"] for b in rep["buckets"]) + 1e-6
        assert rep["bus_GBps"] is not None and rep["bus_GBps"] > 0
        assert rep["comm_exposed_ms"] >= 0


def test_union_of_intervals():
    from s3od_amd.ddp import GradSync
    assert GradSync._union_ms([(0, 2), (1, 3), (5, 6)]) == 4
    assert GradSync._union_ms([(5, 6), (0, 1)]) == 2
    assert GradSync._union_ms([]) == 0
