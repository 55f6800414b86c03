"""Pin the CPU oracle against the golden vectors produced by the reference itself.

CPU only (no GPU marker).  The oracle is a from-scratch restatement; these fixtures came
from importing the reference's models/unet3d.py + utils/losses.py (make_golden.py).
"""
import numpy as np
import pytest
import torch

from oracle import unet3d_cpu as ref
from tests import golden_util as gu

SHA0 = "30bd43350217be6678086943ef7d085e4c31cd929ca6fda2d4c56ba40fec9416"


def test_init_hash_matches_reference_survey():
    torch.manual_seed(0)
    sd = ref.init_params(5, 1)
    assert len(sd) == 136
    assert gu.sd_hash(sd) == SHA0
    assert sum(v.numel() for k, v in sd.items() if k in ref.param_keys(sd)) == 90311361


@pytest.mark.parametrize("name", list(gu.CASES))
def test_oracle_matches_golden(name):
    g = gu.load(name)
    ncls, n, spatial, lab, loss_kind, lr = gu.CASES[name]
    torch.manual_seed(0)
    sd = ref.init_params(5, ncls)
    assert gu.sd_hash(sd) == str(g["sd_sha256"])
    x, y = gu.batch(name, 0)
    assert abs(float(x.double().sum()) - float(g["input_sum"])) < 1e-6
    assert abs(float(y.double().sum()) - float(g["label_sum"])) < 1e-6
    step = ref.RefStep(sd, lr=lr, loss=loss_kind)
    loss0, logits = step.forward_backward(x, y)
    np.testing.assert_allclose(logits.numpy(), g["logits_train"], rtol=0, atol=2e-5)
    assert abs(float(loss0) - float(g["loss0"])) < 1e-5
    for k in step.keys:
        got = gu.sampled(sd[k].grad, g["g_stride__" + k])
        exp = g["g__" + k]
        scale = max(float(np.abs(exp).max()), 1e-12)
        if k.endswith("conv.0.bias") or k.endswith("conv.3.bias"):
            # pre-BN conv biases: exact gradient is 0, value is rounding noise
            assert np.abs(got).max() < 1e-4
            continue
        np.testing.assert_allclose(got, exp, rtol=0, atol=1e-4 * scale + 1e-7, err_msg=k)
    step.opt.step()
    for k in step.keys:
        if k.endswith("conv.0.bias") or k.endswith("conv.3.bias"):
            continue  # H5: Adam normalises the bias noise into lr-sized updates
        got = gu.sampled(sd[k].detach(), g["p_stride__" + k])
        np.testing.assert_allclose(got, g["p__" + k], rtol=1e-5, atol=1e-6, err_msg=k)
    for k in sd:
        if k.endswith(("running_mean", "running_var", "num_batches_tracked")):
            np.testing.assert_allclose(sd[k].numpy(), g["b__" + k], rtol=1e-5, atol=1e-6, err_msg=k)
    with torch.no_grad():
        le = ref.forward(sd, x, training=False)
    np.testing.assert_allclose(le.numpy(), g["logits_eval"], rtol=0, atol=2e-4)
    x1, y1 = gu.batch(name, 1)
    loss1 = step.step(x1, y1)
    assert abs(loss1 - float(g["loss1"])) < 1e-4


def test_dice_shape_mismatch_raises():
    with pytest.raises(ValueError):
        ref.dice_loss(torch.zeros(1, 1, 2, 2, 2), torch.zeros(1, 2, 2, 2, 2))


@pytest.mark.parametrize("cfg", list(gu.FULL_CFGS))
def test_full_fixtures_pinned(cfg):
    """The full-size fixtures (tests/golden/make_golden_full.py, the reference at configs 2, 4
    and 5) were made from the seed-0 init the engine builds (pcms_amd UNet3D, state-dict
    SHA-256) and from the batch the GPU tests regenerate (checksums)."""
    import pcms_amd  # noqa: F401
    from pcms_amd.models.unet3d import UNet3D
    fx = gu.full_fixture(cfg)
    torch.manual_seed(0)
    m = UNet3D(n_modalities=5, n_classes=1)
    assert gu.sd_hash(m.state_dict()) == str(fx["sd_sha256"]) == SHA0
    x, y = gu.full_batch(cfg)
    assert abs(float(x.double().sum()) - float(fx["input_sum"])) <= 1e-9 * abs(float(fx["input_sum"]))
    assert abs(float(y.double().sum()) - float(fx["label_sum"])) < 1e-6
    n = x.shape[0] * x.shape[2] * x.shape[3] * x.shape[4]
    assert fx["m32_bits"].size == (n + 7) // 8
    assert float(fx["e_auto"]) > 0 and 0.9 < float(fx["agree_auto"]) <= 1.0


@pytest.mark.parametrize("cfg", ["cfg2", "cfg4"])
def test_full_fixture_windows_agree_with_sample(cfg):
    """The dense logit planes (make_golden_full.py add_windows: a second run of the reference's
    forward) hold the same numbers as the strided sample of the original step where the two
    meet: the d = 0 plane of sample 0 is flat[0 : H W], the sample's first H W / stride
    entries."""
    fx = gu.full_fixture(cfg)
    ls = int(fx["logit_stride"])
    _, (D, H, W), _ = gu.FULL_CFGS[cfg]
    assert int(fx["win_axis"][0]) == 2 and int(fx["win_index"][0]) == 0
    for tag in ("32", "bf"):
        plane = fx[f"w{tag}__0"][:H * W]          # sample 0, d = 0
        np.testing.assert_array_equal(plane[::ls], fx[f"l{tag}_s"][:(H * W + ls - 1) // ls])
    assert len(fx["win_axis"]) == len(fx["win_index"]) == sum(1 for k in fx if k.startswith("w32__"))


def test_dp3_fixture_autocast_run():
    """full_dp3.npz holds the reference's two-rank step under CPU bf16 autocast as well
    (make_golden_full.py add_dp3_autocast): per-replica losses near the fp32 ones, the mean
    autocast gradient at every sampled tensor, rank 0's buffers, and the slab-chunked layers."""
    fx = gu.full_fixture("dp3")
    assert fx["lossesbf"].shape == fx["losses32"].shape == (2,)
    assert np.all(np.abs(fx["lossesbf"] - fx["losses32"]) < 1e-2)
    g32 = [k[5:] for k in fx if k.startswith("g32__")]
    assert g32 and all("gbf__" + k in fx and fx["gbf__" + k].shape == fx["g32__" + k].shape for k in g32)
    assert all("bbf__" + k[3:] in fx for k in fx if k.startswith("b__"))
    assert "inc.conv.0" in list(fx["autocast_chunked"])
