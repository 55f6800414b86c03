"""Input pipeline (reference script/data_loader.py): NIfTI-1 reader,
ITK-geometry resampling and the ProstateDataset missing-modality strategies.  SimpleITK is
absent, so the resampler is pinned by closed-form cases only (parity unpinned otherwise)."""
import os

import numpy as np
import pytest
import torch


def _data():
    import pcms_amd  # noqa: F401
    from pcms_amd import data
    return data


@pytest.mark.parametrize("ext", [".nii", ".nii.gz"])
@pytest.mark.parametrize("dtype", [np.float32, np.int16, np.uint8])
def test_nifti_roundtrip(tmp_path, ext, dtype):
    d = _data()
    a = (np.random.default_rng(0).random((6, 5, 4)) * 100).astype(dtype)
    p = str(tmp_path / ("v" + ext))
    d.write_nifti(p, a, spacing=(0.5, 0.7, 3.0))
    h = d.read_nifti_header(p)
    assert h["shape_xyz"] == (4, 5, 6) and h["spacing"] == pytest.approx((0.5, 0.7, 3.0))
    b = d.read_nifti(p)
    assert b.shape == a.shape and np.array_equal(b, a)


def test_nifti_scaling_and_4d(tmp_path):
    d = _data()
    import struct
    a = np.arange(2 * 3 * 4 * 5, dtype=np.int16).reshape(2, 3, 4, 5)
    p = str(tmp_path / "s.nii")
    d.write_nifti(p, a)
    with open(p, "r+b") as f:  # scl_slope 2, scl_inter -1
        f.seek(112)
        f.write(struct.pack("<ff", 2.0, -1.0))
    b = d.read_nifti(p)
    assert np.allclose(b, a * 2.0 - 1.0)
    with pytest.raises(ValueError):
        bad = str(tmp_path / "bad.nii")
        open(bad, "wb").write(b"\0" * 400)
        d.read_nifti_header(bad)


def test_resample_closed_forms():
    d = _data()
    rng = np.random.default_rng(1)
    v = rng.random((8, 6, 4)).astype(np.float32)
    assert np.array_equal(d.resample(v, (8, 6, 4)), v)
    # integer down-sampling samples the even voxels exactly
    assert np.allclose(d.resample(v, (4, 3, 2)), v[::2, ::2, ::2])
    # a linear ramp is reproduced by linear up-sampling where it is interpolated
    z = np.arange(8, dtype=np.float32)[:, None, None] * np.ones((1, 2, 2), np.float32)
    up = d.resample(z, (16, 2, 2))
    assert np.allclose(up[:15, 0, 0], np.arange(15) * 0.5)
    assert up[15, 0, 0] == 0.0  # continuous index 7.5 is past the buffer (ITK: default value 0)
    # nearest keeps labels discrete
    lab = (rng.random((8, 8, 8)) > 0.5).astype(np.uint8)
    r = d.resample(lab, (5, 11, 8), nearest=True)
    assert set(np.unique(r)) <= {0.0, 1.0} and r.shape == (5, 11, 8)
    assert np.array_equal(d.resample(lab, (4, 4, 4), nearest=True), lab[::2, ::2, ::2])


def _make_tree(root, cases, target=(8, 8, 8)):
    d = _data()
    rng = np.random.default_rng(2)
    for cid, (mods, has_label, shape) in cases.items():
        for m in mods:
            os.makedirs(os.path.join(root, "BPH-PCA", "BPH", m), exist_ok=True)
            d.write_nifti(os.path.join(root, "BPH-PCA", "BPH", m, cid + ".nii.gz"),
                          (rng.random(shape) * 10).astype(np.float32))
        if has_label:
            ld = os.path.join(root, "BPH-PCA", "ROI(BPH+PCA)", "BPH")
            os.makedirs(ld, exist_ok=True)
            lab = np.zeros(shape, np.uint8)
            lab[2:5, 2:5, 2:5] = 2
            d.write_nifti(os.path.join(ld, cid + ".nii"), lab)


def test_dataset_strategies(tmp_path):
    d = _data()
    mods = d.DEFAULT_MODALITIES
    cases = {"full": (mods, True, (8, 8, 8)),
             "noDWI": ([m for m in mods if m != "DWI"], True, (16, 8, 4)),
             "nolabel": (mods, False, (8, 8, 8))}
    _make_tree(str(tmp_path), cases)
    zf = d.ProstateDataset(str(tmp_path), target_size=(8, 8, 8))
    assert [c["case_id"] for c in zf.case_list] == ["full", "noDWI"]
    s = zf[1]
    assert s["image"].shape == (5, 8, 8, 8) and s["label"].shape == (1, 8, 8, 8)
    assert torch.count_nonzero(s["image"][1]) == 0          # DWI zero-filled
    assert set(torch.unique(s["label"]).tolist()) <= {0.0, 1.0}
    sk = d.ProstateDataset(str(tmp_path), missing_strategy="skip", target_size=(8, 8, 8))
    assert [c["case_id"] for c in sk.case_list] == ["full"]
    du = d.ProstateDataset(str(tmp_path), missing_strategy="duplicate", target_size=(8, 8, 8))
    s = du[1]
    assert torch.equal(s["image"][1], s["image"][0])        # DWI <- ADC (first available)
    with pytest.raises(ValueError):
        d.ProstateDataset(str(tmp_path), missing_strategy="interpolate")
    dl = d.get_dataloader(str(tmp_path), batch_size=2, shuffle=False, target_size=(8, 8, 8))
    b = next(iter(dl))
    assert b["image"].shape == (2, 5, 8, 8, 8) and b["case_id"] == ["full", "noDWI"]


@pytest.mark.parametrize("n,bs,world", [(5, 2, 2), (7, 3, 4), (4, 2, 2), (1, 2, 2)])
def test_eval_batches_shard_without_padding(n, bs, world):
    """Data-parallel evaluation: the ranks' batches are exactly the single-process batches
    (whole, in order, none duplicated), so (sum, count) of per-batch losses over ranks gives
    the reference's validate_epoch mean (DistributedSampler padded the set)."""
    d = _data()
    single = [list(range(lo, min(n, lo + bs))) for lo in range(0, n, bs)]
    got = []
    for r in range(world):
        s = d.BatchShard(n, bs, r, world)
        b = list(s)
        assert len(b) == len(s)
        got += b
    assert sorted(got) == sorted(single)
