"""Checkpoint compatibility (reference utils/trainer.py:236-278,
script/validate_model.py:174-180, script/predict.py:139-145): both checkpoint forms load,
and a saved run resumes with model, Adam and ReduceLROnPlateau state intact."""
import os

import pytest
import torch


def _model(seed):
    import pcms_amd  # noqa: F401
    from pcms_amd.models.unet3d import UNet3D
    torch.manual_seed(seed)
    return UNet3D(n_modalities=5, n_classes=1)


def test_load_weights_both_forms(tmp_path):
    from pcms_amd.models.unet3d import load_weights
    src = _model(0)
    sd = src.state_dict()
    full = {"epoch": 3, "model_state_dict": sd, "optimizer_state_dict": {"state": {}, "param_groups": []},
            "scheduler_state_dict": {}, "loss": 0.5, "config": {"learning_rate": 1e-4}}
    torch.save(full, tmp_path / "latest_checkpoint.pth")
    torch.save(sd, tmp_path / "best_model_epoch_3.pth")
    for name in ("latest_checkpoint.pth", "best_model_epoch_3.pth"):
        dst = _model(1)
        assert not torch.equal(dst.inc.conv[0].weight, src.inc.conv[0].weight)
        load_weights(dst, str(tmp_path / name))
        for k, v in dst.state_dict().items():
            assert torch.equal(v, sd[k]), (name, k)
    dst = _model(1)
    load_weights(dst, full)  # an already loaded dict
    assert torch.equal(dst.outc.weight, src.outc.weight)


@pytest.mark.gpu
def test_trainer_resume_roundtrip(tmp_path):
    from pcms_amd.utils.trainer import Trainer
    cfg = {"device": "cuda", "learning_rate": 1e-4, "batch_size": 2, "num_epochs": 1, "loss": "bce_dice",
           "precision": "fp32", "save_dir": str(tmp_path)}
    gen = torch.Generator().manual_seed(5)
    batches = [{"image": torch.rand(2, 5, 32, 32, 32, generator=gen),
                "label": (torch.rand(2, 1, 32, 32, 32, generator=gen) < 0.3).float()} for _ in range(3)]
    torch.manual_seed(0)
    a = Trainer(cfg)
    a.step(batches[0])
    a.step(batches[1])
    a.scheduler.step(0.7)
    a.save_checkpoint(2, 0.7)
    assert os.path.exists(tmp_path / "latest_checkpoint.pth")
    torch.manual_seed(123)  # different init: everything must come from the file
    b = Trainer(cfg)
    epoch, loss = b.load_checkpoint(str(tmp_path / "latest_checkpoint.pth"))
    assert (epoch, loss) == (2, 0.7)
    for k, v in a.model.state_dict().items():
        assert torch.equal(v, b.model.state_dict()[k]), k
    sa, sb = a.optimizer.state_dict(), b.optimizer.state_dict()
    for i in sa["state"]:
        for f in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sa["state"][i][f], sb["state"][i][f]), (i, f)
        assert float(sa["state"][i]["step"]) == float(sb["state"][i]["step"]) == 2.0
    assert b.scheduler.state_dict() == a.scheduler.state_dict()
    # the resumed run continues bit for bit (every reduction sums in a fixed order)
    la, lb = a.step(batches[2]), b.step(batches[2])
    assert la == lb, (la, lb)
    for (k, pa), pb in zip(a.model.named_parameters(), b.model.parameters()):
        assert torch.equal(pa, pb), k
