"""Host-side pieces of the predict pipeline (script/predict.py:20-100) that need no GPU:
modality loading, min-max normalisation, missing-modality strategies, preprocessing; and
the product's refusal to run on the CPU."""
import numpy as np
import pytest
import torch


def _case(tmp_path, missing=("T2 fs",)):
    from pcms_amd.data import write_nifti
    from pcms_amd.predict import MODALITIES
    rng = np.random.default_rng(1)
    case = tmp_path / "case"
    for i, mod in enumerate(MODALITIES):
        (case / mod).mkdir(parents=True)
        if mod not in missing:
            write_nifti(str(case / mod / "x.nii"), rng.random((4, 5, 6), dtype=np.float32) * 50 - 10)
    return case


def test_load_and_normalise(tmp_path):
    from pcms_amd.predict import load_multimodal_images, preprocess_image
    img, names = load_multimodal_images(str(_case(tmp_path)))
    assert img.shape == (5, 4, 5, 6) and img.dtype == np.float32
    for c in (0, 1, 2, 4):
        assert img[c].min() == 0.0 and img[c].max() == pytest.approx(1.0)
    assert not img[3].any()
    assert preprocess_image(img).shape == (1, 5, 4, 5, 6)


def test_missing_strategies(tmp_path):
    from pcms_amd.predict import load_multimodal_images
    case = _case(tmp_path, missing=("ADC", "DWI"))
    # zero fill before any modality was read uses a (64, 64, 64) volume, which cannot stack
    # with the (4, 5, 6) ones read later: the reference's np.stack raises the same ValueError
    with pytest.raises(ValueError):
        load_multimodal_images(str(case))
    with pytest.raises(FileNotFoundError):
        load_multimodal_images(str(case), handle_missing="skip")
    case2 = _case(tmp_path / "b", missing=("T2 not fs",))
    img2, _ = load_multimodal_images(str(case2), handle_missing="duplicate")
    np.testing.assert_array_equal(img2[4], img2[0])


def test_no_cpu_path():
    from pcms_amd.models.unet3d import DoubleConv3D
    m = DoubleConv3D(8, 64)
    with pytest.raises(RuntimeError):
        m(torch.zeros(1, 8, 4, 4, 4))
