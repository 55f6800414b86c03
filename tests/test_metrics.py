"""Validation metrics (reference script/validate_model.py:24-80) and the GPU evaluation loop."""
import pytest
import torch


def test_dice_iou_values():
    import pcms_amd  # noqa: F401
    from pcms_amd.utils.metrics import calculate_dice_score, calculate_iou
    p = torch.tensor([1, 1, 0, 0, 1.0])
    t = torch.tensor([1, 0, 0, 1, 1.0])
    assert calculate_dice_score(p, t) == pytest.approx(2 * 2 / 6)
    assert calculate_iou(p, t) == pytest.approx(2 / 4)
    z = torch.zeros(8)
    assert calculate_dice_score(z, z) == 0.0 and calculate_iou(z, z) == 0.0
    assert calculate_dice_score(t, t) == pytest.approx(1.0)


@pytest.mark.gpu
def test_evaluate_loop_matches_inference_masks():
    from pcms_amd.models.unet3d import UNet3D
    from pcms_amd.utils.metrics import calculate_dice_score, evaluate
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1).cuda()
    gen = torch.Generator().manual_seed(3)
    batches = [{"image": torch.rand(2, 5, 32, 32, 16, generator=gen),
                "label": (torch.rand(2, 1, 32, 32, 16, generator=gen) < 0.5).float(), "case_id": ["a", "b"]}]
    m.train()
    m(batches[0]["image"].cuda())  # one training forward: running stats move off their init
    r = evaluate(m, batches)
    assert [c["case_id"] for c in r["cases"]] == ["a", "b"]
    mask = m.inference(batches[0]["image"].cuda())
    d0 = calculate_dice_score(mask[0], batches[0]["label"][0].cuda())
    assert r["cases"][0]["dice"] == pytest.approx(d0)
    assert 0.0 <= r["mean_iou"] <= r["mean_dice"] <= 1.0
