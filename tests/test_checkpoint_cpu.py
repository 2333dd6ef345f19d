"""Checkpoint interoperability on CPU (no kernel launches): Lightning-layout save / load of model
weights, FusedAdamW state <-> torch.optim.AdamW state, clean export
(reference: scripts/export_model.py:27-119, src/s3od/predictor.py:65-76)."""
import torch

from s3od_amd.checkpoint import save_checkpoint, load_checkpoint, export_checkpoint, read_checkpoint
from s3od_amd.model import DPTSegmentation
from s3od_amd.optim import FusedAdamW, reference_param_groups


def _fake_adam_state(opt, step=3):
    for g in opt.param_groups:
        for p in g["params"]:
            st = opt.state[p]
            st["step"] = torch.tensor(float(step))
            st["exp_avg"] = torch.full_like(p, 0.25)
            st["exp_avg_sq"] = torch.full_like(p, 0.5)


def test_lightning_ckpt_roundtrip(tmp_path):
    torch.manual_seed(0)
    m = DPTSegmentation()
    opt = FusedAdamW(reference_param_groups(m, 1e-5), weight_decay=0.05)
    _fake_adam_state(opt)
    sch = torch.optim.lr_scheduler.LinearLR(opt, start_factor=1.0, end_factor=1.0, total_iters=30)
    sch.step()
    path = tmp_path / "last.ckpt"
    save_checkpoint(path, m, opt, sch, epoch=4, global_step=40, config={"model": {"_target_": "x"}})
    ck = read_checkpoint(path)
    assert all(k.startswith("model.") for k in ck["state_dict"])
    assert ck["epoch"] == 4 and ck["hyper_parameters"]["config"]["model"]["_target_"] == "x"

    m2 = DPTSegmentation()
    with torch.no_grad():
        for p in m2.parameters():
            p.zero_()
    opt2 = FusedAdamW(reference_param_groups(m2, 1e-5), weight_decay=0.05)
    sch2 = torch.optim.lr_scheduler.LinearLR(opt2, start_factor=1.0, end_factor=1.0, total_iters=30)
    load_checkpoint(path, m2, opt2, sch2)
    for (k, a), (_, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert torch.equal(a, b), k
    p0 = next(iter(m2.parameters()))
    assert float(opt2.state[p0]["step"]) == 3.0 and torch.all(opt2.state[p0]["exp_avg"] == 0.25)
    assert sch2.last_epoch == sch.last_epoch


def test_state_dict_interchanges_with_torch_adamw():
    m = DPTSegmentation()
    opt = FusedAdamW(reference_param_groups(m, 1e-5), weight_decay=0.05)
    _fake_adam_state(opt, step=7)
    ref = torch.optim.AdamW(reference_param_groups(m, 1e-5), weight_decay=0.05)
    ref.load_state_dict(opt.state_dict())
    back = FusedAdamW(reference_param_groups(m, 1e-5), weight_decay=0.05)
    back.load_state_dict(ref.state_dict())
    p = next(iter(m.parameters()))
    assert float(back.state[p]["step"]) == 7.0
    assert torch.equal(back.state[p]["exp_avg_sq"], opt.state[p]["exp_avg_sq"])


def test_export_clean_checkpoint(tmp_path):
    m = DPTSegmentation()
    save_checkpoint(tmp_path / "a.ckpt", m)
    out = export_checkpoint(tmp_path / "a.ckpt", tmp_path / "s3od.pt")
    clean = torch.load(out, map_location="cpu", weights_only=True)
    assert set(clean) == {"state_dict"}
    assert set(clean["state_dict"]) == set(m.state_dict())
    m2 = DPTSegmentation()
    m2.load_state_dict(clean["state_dict"])


def test_export_model_cli(tmp_path):
    """scripts/export_model.py (reference scripts/export_model.py:175-227): --checkpoint/--output/--format."""
    import subprocess
    import sys
    from pathlib import Path
    m = DPTSegmentation(init_seed=None)
    save_checkpoint(tmp_path / "best.ckpt", m, config={"model": {"_target_": "synth_sod.model_training.model.DPTSegmentation"}})
    script = Path(__file__).resolve().parent.parent / "scripts" / "export_model.py"
    r = subprocess.run([sys.executable, str(script), "--checkpoint", str(tmp_path / "best.ckpt"), "--output",
                        str(tmp_path / "s3od.pt")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "contains 371 parameters" in r.stdout
    clean = torch.load(tmp_path / "s3od.pt", map_location="cpu", weights_only=True)
    assert set(clean["state_dict"]) == set(m.state_dict())
    r = subprocess.run([sys.executable, str(script), "--checkpoint", str(tmp_path / "best.ckpt"), "--output",
                        str(tmp_path / "x.pt"), "--format", "torchscript"], capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "TorchScript" in r.stderr
