"""Training launcher: the MI355X equivalent of ``synth_sod/model_training/train.py:72-142``.

Plain torch in place of Hydra + Lightning (neither is in this image):

* ``compose_config(config_dir, overrides)`` reads the reference's own YAML tree (``train.yaml`` with
  its ``defaults`` list of backend / dataset / loss / model / optimizer / scheduler / train_stage
  groups), applies ``group=option`` and ``a.b=value`` overrides and resolves ``${a.b}`` and
  ``${eval:'...'}`` interpolations (train.py:20 registers ``eval``);
* ``fit(config)`` is ``train()``: seeding (``pl.seed_everything(backend.seed)``), the folder datasets
  (``create_dataloaders``, dataset.py:325-425) with a ``DistributedSampler`` per rank and the
  augmentation on device, ``SegmentationLightningModule``, one process per GPU (``backend.devices``;
  spawned through ``torch.distributed.run`` when not already launched) with ``GradSync`` (RCCL
  all-reduce overlapped with the native backward; ``no_sync`` on accumulation micro-batches),
  ``accumulate_grad_batches`` (loss / k, optimizer step every k micro-batches and at the epoch end),
  the LR scheduler stepped once per epoch, a validation pass per epoch with epoch-mean logs
  (``val_dice_epoch`` ...), ``ModelCheckpoint(monitor="val_dice_epoch", mode="max", save_top_k=3,
  save_last=True)``, ``EarlyStopping(**train_stage.early_stopping)`` and resume from
  ``train_stage.checkpoint_path`` (full state, or weights only when ``train_stage.weights_only``).

Lightning / torch DDP strategies are refused: the native backward writes gradients straight into a
flat buffer that only ``GradSync`` exchanges (``SegmentationLightningModule._check_grad_sync``).
Out of scope (tier framing): TensorBoard / image logging, the post-fit evaluation callback.
"""
from __future__ import annotations

import contextlib
import math
import os
import random
import re
import sys
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

# ------------------------------------------------------------------------------------ config
_REF = re.compile(r"\$\{([^{}]+)\}")


def _set(d, dotted, value):
    keys = dotted.split(".")
    for k in keys[:-1]:
        d = d.setdefault(k, {})
    d[keys[-1]] = value


def _get(d, dotted):
    for k in dotted.split("."):
        d = d[k]
    return d


def _loader():
    """yaml.SafeLoader with OmegaConf's float rule (``1e-5`` is a float, as the reference's
    ``optimizer.lr * 10`` requires; plain YAML 1.1 reads it as a string)."""
    import yaml

    class L(yaml.SafeLoader):
        pass
    L.add_implicit_resolver(
        "tag:yaml.org,2002:float",
        re.compile(r"""^(?:[-+]?(?:[0-9][0-9_]*)\.[0-9_]*(?:[eE][-+]?[0-9]+)?
                    |[-+]?(?:[0-9][0-9_]*)(?:[eE][-+]?[0-9]+)
                    |\.[0-9_]+(?:[eE][-+][0-9]+)?
                    |[-+]?\.(?:inf|Inf|INF)
                    |\.(?:nan|NaN|NAN))$""", re.X),
        list("-+0123456789."))
    return L


def _load(text_or_file):
    import yaml
    return yaml.load(text_or_file, Loader=_loader())   # SafeLoader subclass: executes nothing


def _parse_scalar(v):
    return _load(v) if isinstance(v, str) else v


def _resolve(node, root):
    if isinstance(node, dict):
        return {k: _resolve(v, root) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v, root) for v in node]
    if not isinstance(node, str) or "${" not in node:
        return node
    for _ in range(16):                      # innermost interpolations first
        m = _REF.search(node)
        if m is None:
            break
        expr = m.group(1)
        if expr.startswith("eval:"):
            val = eval(expr[5:].strip().strip("'\""), {"__builtins__": {}}, {})   # noqa: S307 (train.py:20)
        elif expr.startswith("now:"):
            import time
            val = time.strftime(expr[4:])
        else:
            val = _resolve(_get(root, expr), root)
        if m.group(0) == node:
            return val
        node = node[:m.start()] + str(val) + node[m.end():]
    return _parse_scalar(node)


def compose_config(config_dir, overrides=(), config_name="train"):
    """Hydra-style composition of the reference's config tree (synth_sod/.../model_training/config)."""
    config_dir = Path(config_dir)
    main = _load(open(config_dir / f"{config_name}.yaml")) or {}
    main.pop("hydra", None)
    defaults = main.pop("defaults", [])
    groups = {}
    for d in defaults:
        if isinstance(d, dict):
            groups.update(d)
    plain = []
    for o in overrides:
        k, v = o.split("=", 1)
        if "." not in k and k in groups:
            groups[k] = v
        else:
            plain.append((k, v))
    cfg = {}
    for g, opt in groups.items():
        cfg[g] = _load(open(config_dir / g / f"{opt}.yaml")) or {}
    cfg.update(main)
    for k, v in plain:
        _set(cfg, k, _parse_scalar(v))
    return _resolve(cfg, cfg)


# ------------------------------------------------------------------------------------ pieces
def seed_everything(seed):
    """pl.seed_everything: python, numpy and torch (all devices) generators."""
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)


def build_loaders(ds_cfg, seed, rank, world):
    """create_dataloaders (dataset.py:325-425) with DistributedSampler (what Lightning injects)."""
    from torch.utils.data import ConcatDataset, DataLoader
    from torch.utils.data.distributed import DistributedSampler
    from .data import MaskDataset
    paths = ds_cfg["datasets"]
    S = int(ds_cfg["image_size"])
    mk = lambda split, mode: [MaskDataset(p, S, split=split, val_split=ds_cfg.get("val_split", 0.1), transform_mode=mode,
                                          seed=seed, debug_subset_fraction=ds_cfg.get("debug_subset_fraction"))
                              for p in paths]
    tr, va = mk("train", ds_cfg.get("transform_mode", "regular")), mk("val", "test")
    tr = tr[0] if len(tr) == 1 else ConcatDataset(tr)
    va = va[0] if len(va) == 1 else ConcatDataset(va)
    nw = int(ds_cfg.get("num_workers", 0))
    ts = DistributedSampler(tr, num_replicas=world, rank=rank, shuffle=True, seed=seed, drop_last=True)
    vs = DistributedSampler(va, num_replicas=world, rank=rank, shuffle=False, drop_last=False)
    kw = dict(num_workers=nw, collate_fn=MaskDataset.collate, persistent_workers=False)
    train_loader = DataLoader(tr, batch_size=int(ds_cfg["train_batch_size"]), sampler=ts, drop_last=True, **kw)
    val_loader = DataLoader(va, batch_size=int(ds_cfg["val_batch_size"]), sampler=vs, drop_last=False, **kw)
    return train_loader, val_loader


class TopK:
    """ModelCheckpoint(dirpath, filename="{epoch:02d}-{val_dice_epoch:.4f}", monitor, mode, save_top_k, save_last)."""

    def __init__(self, dirpath, monitor="val_dice_epoch", mode="max", k=3, save_last=True):
        self.dir = Path(dirpath)
        self.monitor, self.mode, self.k, self.save_last = monitor, mode, k, save_last
        self.best = []           # (score, path)
        self.best_model_path = None

    def _better(self, a, b):
        return a > b if self.mode == "max" else a < b

    def update(self, epoch, metrics, save_fn):
        self.dir.mkdir(parents=True, exist_ok=True)
        if self.save_last:
            save_fn(self.dir / "last.ckpt")
        score = metrics.get(self.monitor)
        if score is None or not math.isfinite(score):
            return
        if len(self.best) < self.k or self._better(score, self.best[-1][0]):
            path = self.dir / f"epoch={epoch:02d}-{self.monitor}={score:.4f}.ckpt"
            save_fn(path)
            self.best.append((score, path))
            self.best.sort(key=lambda t: -t[0] if self.mode == "max" else t[0])
            while len(self.best) > self.k:
                _, old = self.best.pop()
                if old.exists():
                    old.unlink()
            self.best_model_path = str(self.best[0][1])


class EarlyStop:
    def __init__(self, monitor, min_delta=0.0, patience=3, mode="min"):
        self.monitor, self.min_delta, self.patience, self.mode = monitor, float(min_delta), int(patience), mode
        self.best, self.wait = None, 0

    def should_stop(self, metrics):
        v = metrics.get(self.monitor)
        if v is None:
            return False
        improved = self.best is None or (v < self.best - self.min_delta if self.mode == "min" else v > self.best + self.min_delta)
        if improved:
            self.best, self.wait = v, 0
        else:
            self.wait += 1
        return self.wait >= self.patience


def _epoch_means(acc):
    return {f"{k}_epoch": s / n for k, (s, n) in acc.items() if n > 0}


def _accumulate(acc, logs, weight):
    for k, v in logs.items():
        s, n = acc.get(k, (0.0, 0))
        acc[k] = (s + float(v) * weight, n + weight)


# ------------------------------------------------------------------------------------ fit
def fit(config, train_loader=None, val_loader=None, augment=None, val_augment=None, log=print):
    """train.py:72-142.  Returns a summary dict (epochs run, optimizer steps, best checkpoint, last metrics)."""
    from .lightning_module import SegmentationLightningModule
    from .checkpoint import save_checkpoint, load_checkpoint
    from .data import GpuAugment
    from .ddp import GradSync, broadcast_parameters

    be, ds, ts = config["backend"], config["dataset"], config["train_stage"]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if world > 1 and not dist.is_initialized():
        # a rank that stops answering (hung kernel, dead peer) fails the collective after this long
        # instead of hanging the job: TORCH_NCCL_ASYNC_ERROR_HANDLING aborts the communicator
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        dist.init_process_group("nccl", device_id=dev, timeout=rccl_timeout())
    seed = int(be.get("seed", 42))
    seed_everything(seed)
    if train_loader is None:
        train_loader, val_loader = build_loaders(ds, seed, rank, world)
    S = int(ds["image_size"])
    augment = augment or GpuAugment(S, mode=ds.get("transform_mode", "regular"), device=dev)
    val_augment = val_augment or GpuAugment(S, mode="test", device=dev)

    module = SegmentationLightningModule(config).to(dev)
    model = module.model
    sync = None
    if world > 1:
        broadcast_parameters(model)
        sync = GradSync(model)
    opt_cfg = module.configure_optimizers()
    opt = opt_cfg["optimizer"]
    sched = opt_cfg.get("lr_scheduler", {}).get("scheduler")
    accum = int(be.get("accumulate_grad_batches", 1))
    max_epochs = int(be.get("max_epochs", 1))
    start_epoch, global_step = 0, 0
    ckpt_path = ts.get("checkpoint_path")
    if ckpt_path:
        if ts.get("weights_only", False):
            load_checkpoint(ckpt_path, module)
        else:
            ck = load_checkpoint(ckpt_path, module, optimizer=opt, scheduler=sched)
            start_epoch = int(ck.get("epoch", 0)) + 1
            global_step = int(ck.get("global_step", 0))
    # get_experiment_name (train.py:58-69): <experiment_name>_<timestamp>, so a second run with the same
    # name never mixes its top-k files with an earlier run's; rank 0 (the only writer) picks the stamp
    name = experiment_dir_name(ts.get("experiment_name", "s3od"))
    topk = TopK(Path(ts.get("save_dir", "checkpoints")) / name, monitor="val_dice_epoch", mode="max", k=3, save_last=True)
    es_cfg = ts.get("early_stopping")
    stopper = EarlyStop(**es_cfg) if es_cfg else None
    history = []
    epoch = start_epoch - 1
    # non-finite loss guard: counted on device every micro-step, checked (one sync) every
    # `nan_check_every` steps and at each epoch end -> FloatingPointError naming the step
    nan_every = int(be.get("nan_check_every", 50))
    bad = torch.zeros((), dtype=torch.int32, device=dev)

    def check_finite(where):
        nan_guard(bad, world, where)
    for epoch in range(start_epoch, max_epochs):
        module.current_epoch_ = epoch
        if hasattr(train_loader, "sampler") and hasattr(train_loader.sampler, "set_epoch"):
            train_loader.sampler.set_epoch(epoch)
        model.train()
        acc = {}
        nb = len(train_loader)
        for i, samples in enumerate(train_loader):
            batch = augment(samples) if augment is not None and isinstance(samples, list) else samples
            last_micro = (i + 1) % accum == 0 or i + 1 == nb
            ctx = sync.no_sync() if (sync is not None and not last_micro) else contextlib.nullcontext()
            with ctx:
                loss = module.training_step(batch, i)
                (loss / accum).backward()
            bad += (~torch.isfinite(loss.detach())).to(torch.int32)
            if nan_every > 0 and (i + 1) % nan_every == 0:
                check_finite(f"epoch {epoch} batch {i}")
            logs = module.flush_logs()
            _accumulate(acc, logs, batch["images"].shape[0])
            if last_micro:
                opt.step()
                model.zero_grad(set_to_none=False)
                global_step += 1
        check_finite(f"the end of epoch {epoch}")
        metrics = _epoch_means(acc)
        if val_loader is not None:
            model.eval()
            vacc = {}
            with torch.no_grad():
                for i, samples in enumerate(val_loader):
                    batch = val_augment(samples) if isinstance(samples, list) else samples
                    module.validation_step(batch, i)
                    _accumulate(vacc, module.flush_logs(), batch["images"].shape[0])
            metrics.update(_epoch_means(vacc))
        if sched is not None:
            sched.step()
        metrics["lr"] = [g["lr"] for g in opt.param_groups]
        history.append(dict(epoch=epoch, global_step=global_step, **metrics))
        if rank == 0:
            log(f"epoch {epoch}: " + ", ".join(f"{k}={v:.5g}" for k, v in metrics.items() if isinstance(v, float)))
            topk.update(epoch, metrics, lambda p: save_checkpoint(p, module, opt, sched, epoch=epoch, global_step=global_step,
                                                                  config=config))
        if stopper is not None and stopper.should_stop(metrics):
            break
    if world > 1:
        dist.barrier()
    evaluation = None
    ev = ts.get("evaluation") or {}
    if rank == 0 and ev.get("enabled") and topk.best_model_path:
        evaluation = evaluate(ev, topk.best_model_path, log)
    return {"epochs": epoch + 1 - start_epoch, "global_step": global_step, "best_model_path": topk.best_model_path,
            "history": history, "module": module, "optimizer": opt, "scheduler": sched, "evaluation": evaluation}


def experiment_dir_name(base, now=None):
    """get_experiment_name (train.py:58-69): ``f"{base}_{%Y%m%d_%H%M%S}"``."""
    import datetime
    return f"{base}_{(now or datetime.datetime.now()).strftime('%Y%m%d_%H%M%S')}"


def nan_guard(bad, world, where, group=None):
    """Raise FloatingPointError when any rank counted a non-finite loss.  The per-rank counter is
    MAX-all-reduced first, so every rank takes the same raise/continue decision at the same step (a
    rank raising alone would leave its peers blocked in the next collective until the timeout)."""
    if world > 1:
        flag = bad.clone()
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
    else:
        flag = bad
    n = int(flag)
    if n > 0:
        raise FloatingPointError(f"non-finite training loss ({n} micro-batches on the worst rank) before {where}")


def rccl_timeout():
    """Collective timeout (S3OD_RCCL_TIMEOUT_S, default 30 min, as torch.distributed's default)."""
    import datetime
    return datetime.timedelta(seconds=int(os.environ.get("S3OD_RCCL_TIMEOUT_S", "1800")))


def evaluate(ev, best_model_path, log=print):
    """train.py:24-55 EvaluationCallback.on_fit_end: score the best checkpoint on every test dataset
    with SODPredictor + the device metrics (compute_metrics.process_dataset)."""
    from .metrics import process_dataset
    from .sod_predictor import SODPredictor
    predictor = SODPredictor(best_model_path, int(ev.get("image_size", 1024)), device="cuda")
    out = {}
    for name in ev.get("datasets") or []:
        out[name] = process_dataset(os.path.join(str(ev["input_dir"]), name), predictor)
        log(f"\n{name} metrics:")
        log(out[name])
    return out


def dry_run(cfg):
    """The launch path without a GPU: every rank joins a gloo group, the ranks all-reduce their rank ids and
    their DistributedSampler shard sizes, and rank 0 prints one JSON line (world size, devices requested)."""
    import json
    from torch.utils.data.distributed import DistributedSampler
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo", timeout=rccl_timeout())
    bs = int(cfg["dataset"].get("train_batch_size", 1))
    n = 10 * bs * max(world, 1) + 3                              # a ragged synthetic dataset length
    shard = len(DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=True, drop_last=True))
    t = torch.tensor([float(rank), float(shard), 1.0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"dry_run": True, "world_size": world, "devices": int(cfg["backend"].get("devices", 1)),
                          "rank_sum": int(t[0]), "samples_per_epoch": int(t[1]), "ranks_joined": int(t[2]),
                          "accumulate_grad_batches": int(cfg["backend"].get("accumulate_grad_batches", 1))}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


def main(argv=None):
    """``python -m s3od_amd.train --config-dir <synth_sod/.../config> backend=8gpu dataset=synth ...``"""
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-dir", required=True)
    ap.add_argument("--config-name", default="train")
    ap.add_argument("--dry-run", action="store_true",
                    help="spawn the ranks and join a gloo group (no GPU call), report the world from rank 0, exit")
    ap.add_argument("overrides", nargs="*")
    args = ap.parse_args(argv)
    cfg = compose_config(args.config_dir, args.overrides, args.config_name)
    devices = int(cfg["backend"].get("devices", 1))
    if devices > 1 and "WORLD_SIZE" not in os.environ:
        import subprocess
        import socket
        s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={devices}",
               "--master-addr=127.0.0.1", f"--master-port={port}", "-m", "s3od_amd.train"] + list(argv or sys.argv[1:])
        return subprocess.call(cmd)
    if args.dry_run:
        return dry_run(cfg)
    out = fit(cfg)
    print({k: v for k, v in out.items() if k in ("epochs", "global_step", "best_model_path")})
    return 0


if __name__ == "__main__":
    sys.exit(main())
