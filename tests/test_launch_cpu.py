"""CPU: the multi-rank launch paths, without a GPU.  `python bench.py --gpus 2 --dry-run` and
`python -m s3od_amd.train ... backend.devices=2 --dry-run` each spawn two ranks under
torch.distributed.run (the same child-process launch the timed run uses), every rank joins a gloo group
before any GPU call, and rank 0 reports world_size 2 (the reference launches its ranks through
Lightning's `devices` = backend/8gpu.yaml:1-6, train.py:116-125)."""
import json
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _env():
    env = dict(os.environ)
    env.update(PYTHONPATH=str(ROOT), HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    return env


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out              # rank 0 only
    return json.loads(lines[0])


def test_bench_gpus2_dry_run():
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "2", "--dry-run"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["dry_run"] and d["world_size"] == 2 and d["ranks_joined"] == 2
    assert d["rank_sum"] == 1 and d["local_rank_sum"] == 1          # ranks 0 + 1, local ranks 0 + 1
    assert d["global_batch"] == 32 and d["parallelism"] == "dp2"     # 16 per GPU (weak scaling)


def test_train_devices2_dry_run(tmp_path):
    for g, body in {"backend": "devices: 2\naccumulate_grad_batches: 16\nseed: 42\n",
                    "dataset": "train_batch_size: 4\nimage_size: 1024\n"}.items():
        (tmp_path / g).mkdir()
        (tmp_path / g / "x.yaml").write_text(body)
    (tmp_path / "train.yaml").write_text("defaults:\n  - backend: x\n  - dataset: x\n")
    r = subprocess.run([sys.executable, "-m", "s3od_amd.train", "--config-dir", str(tmp_path), "--dry-run"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["dry_run"] and d["world_size"] == 2 and d["devices"] == 2 and d["ranks_joined"] == 2
    assert d["rank_sum"] == 1 and d["accumulate_grad_batches"] == 16
    assert d["samples_per_epoch"] == 2 * ((10 * 4 * 2 + 3) // 2)     # DistributedSampler(drop_last) shards
