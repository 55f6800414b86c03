"""Input pipeline feeding ``Trainer.step`` (reference script/data_loader.py).

The reference reads NIfTI volumes with SimpleITK, which is absent here, so this module has
its own NIfTI-1 reader (``read_nifti``: .nii / .nii.gz, the header's scl_slope/scl_inter
applied, array in SimpleITK ``GetArrayFromImage`` order (z, y, x)) and its own resampler
(``resample``: the reference's ResampleImageFilter set-up — same origin and direction,
output spacing = size * spacing / target, linear for images, nearest for labels).  The
resampler is ITK's index mapping restated (output index i samples input continuous index
i * n_in / n_out); without SimpleITK its results are parity-unpinned beyond the tests'
closed-form cases (identity, integer down-sampling, constant and linear ramps).

Dataset semantics follow script/data_loader.py:
  * case discovery from ``<data_dir>/BPH-PCA/<data_type>/ADC/*.nii[.gz]`` (:57-94);
  * per-modality files ``<data_dir>/BPH-PCA/<data_type>/<modality>/<case>.nii[.gz]``, labels
    ``<data_dir>/BPH-PCA/ROI(BPH+PCA)/<data_type>/<case>.nii[.gz]``; cases without a label or
    with an unreadable header are dropped (:96-194);
  * missing modalities: 'skip' drops the case, 'duplicate' copies the first available
    modality (none available: dropped), 'zero_fill' loads zeros of ``target_size``
    (:147-163, :318-333);
  * every modality resampled (linear) to ``target_size`` (D, H, W), label resampled
    (nearest) and binarised ``> 0`` (:240-283, :379-409);
  * batches ``{'image': (N, M, D, H, W) f32, 'label': (N, 1, D, H, W) f32, 'case_id': [..]}``
    from a ``DataLoader`` with ``pin_memory`` (:421-466).
The reference's SimpleITK ``SetSize`` takes (x, y, z), so its non-cubic outputs come out
axis-reversed; here ``target_size`` is (D, H, W) as documented (:41).
"""
from __future__ import annotations

import glob
import gzip
import os
import struct
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

DEFAULT_MODALITIES = ["ADC", "DWI", "gaoqing-T2", "T2 fs", "T2 not fs"]

# NIfTI-1 datatype codes -> numpy dtypes
_NIFTI_DTYPES = {2: np.uint8, 4: np.int16, 8: np.int32, 16: np.float32, 64: np.float64, 256: np.int8,
                 512: np.uint16, 768: np.uint32, 1024: np.int64, 1280: np.uint64}


def _open(path: str):
    return gzip.open(path, "rb") if path.endswith(".gz") else open(path, "rb")


def read_nifti_header(path: str) -> dict:
    """Parse the 348-byte NIfTI-1 header (either byte order); ValueError if it is not one."""
    with _open(path) as f:
        raw = f.read(348)
    if len(raw) < 348:
        raise ValueError(f"{path}: truncated NIfTI header")
    for endian in ("<", ">"):
        if struct.unpack(endian + "i", raw[:4])[0] == 348:
            break
    else:
        raise ValueError(f"{path}: not a NIfTI-1 file (sizeof_hdr != 348)")
    dim = struct.unpack(endian + "8h", raw[40:56])
    datatype, bitpix = struct.unpack(endian + "hh", raw[70:74])
    pixdim = struct.unpack(endian + "8f", raw[76:108])
    vox_offset, scl_slope, scl_inter = struct.unpack(endian + "fff", raw[108:120])
    magic = raw[344:348]
    if magic not in (b"n+1\x00", b"ni1\x00"):
        raise ValueError(f"{path}: bad NIfTI magic {magic!r}")
    if datatype not in _NIFTI_DTYPES:
        raise ValueError(f"{path}: unsupported NIfTI datatype {datatype}")
    nd = dim[0]
    if not 1 <= nd <= 7:
        raise ValueError(f"{path}: bad dim[0] = {nd}")
    return {"endian": endian, "shape_xyz": tuple(int(d) for d in dim[1:1 + nd]), "datatype": datatype,
            "bitpix": bitpix, "spacing": tuple(float(p) for p in pixdim[1:1 + nd]),
            "vox_offset": int(vox_offset), "scl_slope": float(scl_slope), "scl_inter": float(scl_inter)}


def read_nifti(path: str) -> np.ndarray:
    """Voxel array in SimpleITK ``GetArrayFromImage`` order: (z, y, x), or (t, z, y, x).
    Intensity scaling (scl_slope != 0) is applied, as ITK's NIfTI reader does."""
    h = read_nifti_header(path)
    dt = np.dtype(_NIFTI_DTYPES[h["datatype"]]).newbyteorder(h["endian"])
    count = int(np.prod(h["shape_xyz"]))
    with _open(path) as f:
        f.read(max(h["vox_offset"], 352))
        buf = f.read(count * dt.itemsize)
    if len(buf) < count * dt.itemsize:
        raise ValueError(f"{path}: truncated voxel data")
    arr = np.frombuffer(buf, dtype=dt, count=count).reshape(h["shape_xyz"][::-1])
    if h["scl_slope"] not in (0.0, 1.0) or h["scl_inter"] != 0.0:
        slope = h["scl_slope"] if h["scl_slope"] != 0.0 else 1.0
        arr = arr.astype(np.float64) * slope + h["scl_inter"]
    return np.ascontiguousarray(arr)


def write_nifti(path: str, arr_zyx: np.ndarray, spacing: Sequence[float] = (1.0, 1.0, 1.0)) -> None:
    """Minimal NIfTI-1 writer (single file, little endian) for tests and synthetic data."""
    codes = {np.dtype(v): k for k, v in _NIFTI_DTYPES.items()}
    a = np.ascontiguousarray(arr_zyx)
    if a.dtype not in codes:
        a = a.astype(np.float32)
    a = a.astype(a.dtype.newbyteorder("<"))
    shape_xyz = a.shape[::-1]
    hdr = bytearray(352)
    struct.pack_into("<i", hdr, 0, 348)
    dims = [len(shape_xyz)] + list(shape_xyz) + [1] * (7 - len(shape_xyz))
    struct.pack_into("<8h", hdr, 40, *dims)
    struct.pack_into("<hh", hdr, 70, codes[a.dtype], a.dtype.itemsize * 8)
    pix = [1.0] + list(spacing) + [1.0] * (7 - len(spacing))
    struct.pack_into("<8f", hdr, 76, *pix[:8])
    struct.pack_into("<fff", hdr, 108, 352.0, 1.0, 0.0)
    hdr[344:348] = b"n+1\x00"
    data = bytes(hdr) + a.tobytes()
    with (gzip.open(path, "wb") if path.endswith(".gz") else open(path, "wb")) as f:
        f.write(data)


def _axis_linear(a: np.ndarray, axis: int, n_out: int) -> np.ndarray:
    """ITK linear resampling along one axis: output i samples continuous input index
    c = i * n_in / n_out; neighbours clamped at the border, zero outside [-0.5, n_in - 0.5)."""
    n_in = a.shape[axis]
    if n_in == n_out:
        return a
    c = np.arange(n_out, dtype=np.float64) * (n_in / n_out)
    inside = (c >= -0.5) & (c < n_in - 0.5)
    i0 = np.floor(c).astype(np.int64)
    w = (c - i0).reshape([-1 if d == axis else 1 for d in range(a.ndim)])
    lo = np.clip(i0, 0, n_in - 1)
    hi = np.clip(i0 + 1, 0, n_in - 1)
    out = np.take(a, lo, axis=axis) * (1.0 - w) + np.take(a, hi, axis=axis) * w
    mask = inside.reshape(w.shape)
    return np.where(mask, out, 0.0)


def _axis_nearest(a: np.ndarray, axis: int, n_out: int) -> np.ndarray:
    """ITK nearest neighbour along one axis (index rounded half up)."""
    n_in = a.shape[axis]
    if n_in == n_out:
        return a
    c = np.arange(n_out, dtype=np.float64) * (n_in / n_out)
    idx = np.floor(c + 0.5).astype(np.int64)
    inside = idx < n_in
    out = np.take(a, np.clip(idx, 0, n_in - 1), axis=axis)
    mask = inside.reshape([-1 if d == axis else 1 for d in range(a.ndim)])
    return np.where(mask, out, 0)


def resample(vol: np.ndarray, target: Tuple[int, int, int], nearest: bool = False) -> np.ndarray:
    """Resample a (D, H, W) volume to ``target`` with the reference's ResampleImageFilter
    geometry (script/data_loader.py:258-281 images, linear; :383-406 labels, nearest)."""
    out = vol.astype(np.float64) if not nearest else vol
    f = _axis_nearest if nearest else _axis_linear
    for ax in range(3):
        out = f(out, ax, int(target[ax]))
    return out.astype(np.float32)


def _find(base: str, case_id: str) -> Optional[str]:
    for ext in (".nii", ".nii.gz"):
        p = os.path.join(base, case_id + ext)
        if os.path.exists(p):
            return p
    return None


class ProstateDataset(Dataset):
    """script/data_loader.py:9-419 (same constructor, case filtering and sample dicts)."""

    def __init__(self, data_dir: str, modalities: Optional[List[str]] = None, missing_strategy: str = "zero_fill",
                 target_size: Tuple[int, int, int] = (128, 128, 128), is_training: bool = True,
                 data_type: str = "BPH"):
        if missing_strategy not in ("zero_fill", "skip", "duplicate"):
            raise ValueError(f"unsupported missing-modality strategy: {missing_strategy}")
        self.data_dir = data_dir
        self.modalities = list(modalities or DEFAULT_MODALITIES)
        self.missing_strategy = missing_strategy
        self.target_size = tuple(int(v) for v in target_size)
        self.is_training = is_training
        self.data_type = data_type
        self.case_list = self._filter_cases(self._get_case_list())

    def _root(self, *parts) -> str:
        return os.path.join(self.data_dir, "BPH-PCA", *parts)

    def _get_case_list(self) -> List[str]:
        adc = self._root(self.data_type, "ADC")
        if not os.path.isdir(adc):
            return []
        ids = []
        for p in sorted(glob.glob(os.path.join(adc, "*.nii")) + glob.glob(os.path.join(adc, "*.nii.gz"))):
            name = os.path.basename(p)
            ids.append(name[:-7] if name.endswith(".nii.gz") else name[:-4])
        return ids

    def _filter_cases(self, case_ids: List[str]) -> List[Dict]:
        valid = []
        for cid in case_ids:
            files, missing = {}, []
            for m in self.modalities:
                p = _find(self._root(self.data_type, m), cid)
                if p is None:
                    missing.append(m)
                else:
                    files[m] = p
            label = _find(self._root("ROI(BPH+PCA)", self.data_type), cid)
            if label is None:
                continue
            if missing:
                if self.missing_strategy == "skip":
                    continue
                if self.missing_strategy == "duplicate":
                    avail = [m for m in self.modalities if m not in missing]
                    if not avail:
                        continue
                    for m in missing:
                        files[m] = files[avail[0]]
            try:
                for p in list(files.values()) + [label]:
                    read_nifti_header(p)
            except (ValueError, OSError):
                continue
            valid.append({"case_id": cid, "modality_files": files, "label_path": label,
                          "missing_modalities": missing})
        return valid

    def __len__(self) -> int:
        return len(self.case_list)

    @staticmethod
    def _first_volume(a: np.ndarray) -> np.ndarray:
        if a.ndim == 3:
            return a
        if a.ndim == 4:
            return a[0]
        raise ValueError(f"unsupported image dimensions: {a.shape}")

    def __getitem__(self, idx: int) -> Dict:
        case = self.case_list[idx]
        chans = []
        for m in self.modalities:
            p = case["modality_files"].get(m)
            if p is None:  # zero_fill (duplicate cases have every modality mapped)
                chans.append(np.zeros(self.target_size, dtype=np.float32))
                continue
            vol = self._first_volume(read_nifti(p)).astype(np.float32)
            if vol.shape != self.target_size:
                vol = resample(vol, self.target_size)
            chans.append(vol)
        lab = self._first_volume(read_nifti(case["label_path"]))
        if lab.shape != self.target_size:
            lab = resample(lab, self.target_size, nearest=True)
        label = (lab > 0).astype(np.float32)[None]
        return {"image": torch.from_numpy(np.stack(chans, 0)).float(), "label": torch.from_numpy(label),
                "case_id": case["case_id"]}


def get_dataloader(data_dir: str, batch_size: int = 2, shuffle: bool = True, modalities=None,
                   missing_strategy: str = "zero_fill", target_size=(128, 128, 128), num_workers: int = 0,
                   is_training: bool = True, data_type: str = "BPH", indices=None, rank: int = 0,
                   world_size: int = 1) -> DataLoader:
    """script/data_loader.py:421-466 (pinned host batches; Trainer stages them to the GPU on
    a copy stream one batch ahead).  ``world_size > 1``: each rank iterates its own
    DistributedSampler shard (call ``loader.sampler.set_epoch(epoch)`` every epoch)."""
    ds = ProstateDataset(data_dir, modalities=modalities, missing_strategy=missing_strategy,
                         target_size=target_size, is_training=is_training, data_type=data_type)
    if indices is not None:
        ds = torch.utils.data.Subset(ds, indices)
    sampler = None
    if world_size > 1 and not is_training:
        # evaluation: whole batches of the single-process order, batch b on rank b % W (no
        # padding, no duplicates: the (sum, count) of per-batch losses over ranks is the
        # single-process mean)
        return DataLoader(ds, batch_sampler=BatchShard(len(ds), batch_size, rank, world_size),
                          num_workers=num_workers, pin_memory=torch.cuda.is_available())
    if world_size > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world_size, rank=rank,
                                                                  shuffle=shuffle)
    return DataLoader(ds, batch_size=batch_size, shuffle=shuffle and sampler is None, sampler=sampler,
                      num_workers=num_workers, pin_memory=torch.cuda.is_available())


class BatchShard(torch.utils.data.Sampler):
    """Batches ``b = 0, 1, ...`` of ``range(n)`` in order (``batch_size`` each, the last one
    short), keeping those with ``b % world_size == rank``."""

    def __init__(self, n: int, batch_size: int, rank: int, world_size: int):
        self.n, self.bs, self.rank, self.world = n, batch_size, rank, world_size

    def __iter__(self):
        for b, lo in enumerate(range(0, self.n, self.bs)):
            if b % self.world == self.rank:
                yield list(range(lo, min(self.n, lo + self.bs)))

    def __len__(self):
        nb = -(-self.n // self.bs)
        return max(0, -(-(nb - self.rank) // self.world))

    def set_epoch(self, epoch: int) -> None:  # the evaluation order does not change
        pass


def kfold_indices(n_cases: int, n_splits: int = 5, seed: int = 42):
    """sklearn ``KFold(n_splits, shuffle=True, random_state=seed).split(range(n_cases))``
    restated (the reference's get_kfold_splits, script/data_loader.py:468-497): a legacy
    numpy RandomState(seed) shuffle of arange(n), folds of n // k (+1 for the first n % k),
    each fold's test and train indices in ascending order."""
    if n_splits < 2 or n_splits > n_cases:
        raise ValueError(f"cannot split {n_cases} cases into {n_splits} folds")
    order = np.arange(n_cases)
    np.random.RandomState(seed).shuffle(order)
    sizes = np.full(n_splits, n_cases // n_splits, dtype=int)
    sizes[: n_cases % n_splits] += 1
    splits, cur = [], 0
    for sz in sizes:
        mask = np.zeros(n_cases, dtype=bool)
        mask[order[cur:cur + sz]] = True
        cur += sz
        idx = np.arange(n_cases)
        splits.append((idx[~mask], idx[mask]))
    return splits


def get_kfold_splits(data_dir: str, n_splits: int = 5, modalities=None, missing_strategy: str = "zero_fill",
                     target_size=(128, 128, 128), data_type: str = "BPH"):
    """script/data_loader.py:468-497: K (train_indices, val_indices) pairs over the case list
    scanned from <data_dir>/BPH-PCA/<data_type>/ADC (KFold, shuffle, random_state 42)."""
    ds = ProstateDataset.__new__(ProstateDataset)
    ds.data_dir, ds.data_type = data_dir, data_type
    return kfold_indices(len(ds._get_case_list()), n_splits)
