"""Drop-in ``BaseTrainer`` / ``Trainer`` for utils/trainer.py of the reference.

The per-batch step of utils/trainer.py:179-195 becomes ``Trainer.step(batch) -> float``:

    images, labels -> device      (:179-180)
    optimizer.zero_grad()         (:183)
    outputs = model(images)       (:184)   HIP forward
    loss = criterion(outputs, y)  (:187)   HIP loss
    loss.backward()               (:191)   HIP backward (+ RCCL all-reduce of the flat grads)
    optimizer.step()              (:192)   one flat Adam launch
    return loss.item()            (:188/195, one host sync instead of two)

Data parallel (one process per GPU, ``torch.distributed`` with the "nccl" = RCCL backend):
every rank runs the step on its shard; rank 0's BatchNorm running buffers are broadcast
before the forward (DistributedDataParallel(broadcast_buffers=True) semantics) and the
flat fp32 gradient is summed by a few large bucketed all-reduces that run beside the
backward as it finishes each module (``pcms_amd.dp.GradSync``), the 1/world mean folded
into Adam.
BatchNorm statistics and the global Dice stay per replica (plain BatchNorm3d).

Config keys follow utils/trainer.py:40-49 (``device``, ``learning_rate``, ``batch_size``,
``num_epochs``, ``save_dir``, ``validation`` ...) plus ``loss`` ('dice' | 'bce_dice'),
``precision`` ('bf16' | 'fp32'), ``checkpoint_decoder``, and the step variants of the other
reference trainers:
  ``max_grad_norm``  clip_grad_norm_(max_norm) before Adam (train_bph.py:166,
                     train_bph_cv.py:311 use 1.0): one fused norm pass, the clip coefficient
                     folded into the Adam kernel;
  ``use_amp``        GradScaler loss scaling around the step (train_bph_optimized.py:248-298;
                     see pcms_amd.amp: the reduced-precision engine path is bf16).
With ``data_dir`` the loaders come from ``pcms_amd.data.get_dataloader`` (script/data_loader.py;
a DistributedSampler shard per rank under data parallelism); otherwise pass ``train_loader``
/ ``val_loader`` iterables of batch dicts.
"""
from __future__ import annotations

import math
import os
from typing import Iterable, Optional

import torch
import torch.distributed as dist

from .._lib import call, query
from ..amp import GradScaler
from ..dp import GradSync
from ..models.unet3d import UNet3D
from ..optim import FlatAdam
from .losses import BCEDiceLoss, DiceLoss


class BaseTrainer:
    def __init__(self, config: dict, train_loader: Optional[Iterable] = None,
                 val_loader: Optional[Iterable] = None, model: Optional[UNet3D] = None):
        self.config = config
        self._bw_seed = None  # the backward's ones seed, reused (see step)
        self.device = torch.device(config.get("device", "cuda"))
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        self.distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
        self.world_size = dist.get_world_size() if self.distributed else 1
        self.rank = dist.get_rank() if self.distributed else 0
        self.model = model if model is not None else self._create_model()
        self.criterion = self._create_criterion()
        self.optimizer = self._create_optimizer()
        self.scheduler = self._create_scheduler()
        self.train_loader = train_loader if train_loader is not None else self._create_dataloader("train")
        self.val_loader = val_loader
        if self.val_loader is None and config.get("validation", False):
            self.val_loader = self._create_dataloader("test")
        self._copy_stream = None
        self._sync = None
        self.max_grad_norm = config.get("max_grad_norm", config.get("grad_clip"))
        self.scaler = GradScaler(init_scale=config.get("amp_init_scale", 2.0 ** 16)) if config.get("use_amp") else None
        self._clip_bufs = None
        self.last_grad_norm = None   # device tensor: the total gradient norm of the last clipped step
        self._resume = (float("inf"), 0)   # (best loss, patience) carried by a loaded checkpoint
        if self.distributed:
            self._broadcast_params()
        if config.get("save_dir"):
            os.makedirs(config["save_dir"], exist_ok=True)

    # ---- construction (utils/trainer.py:76-158) ----
    def _create_model(self):
        return UNet3D(n_modalities=self.config.get("n_modalities", 5), n_classes=1,
                      precision=self.config.get("precision", "bf16"),
                      checkpoint_decoder=self.config.get("checkpoint_decoder", False)).to(self.device)

    def _create_criterion(self):
        return BCEDiceLoss() if self.config.get("loss", "dice") == "bce_dice" else DiceLoss()

    def _create_optimizer(self):
        return FlatAdam(self.model, lr=self.config["learning_rate"], weight_decay=1e-5)

    def _create_scheduler(self):
        return torch.optim.lr_scheduler.ReduceLROnPlateau(self.optimizer, mode="min", patience=10, factor=0.5)

    def _create_dataloader(self, mode):
        """utils/trainer.py:139-158 with the arguments get_dataloader actually takes (the
        reference passes ``mode=`` / ``handle_missing_modalities=``, which it rejects); under
        data parallelism each rank reads its own DistributedSampler shard."""
        if self.config.get("data_dir") is None:
            return None
        from ..data import get_dataloader
        return get_dataloader(self.config["data_dir"], batch_size=self.config["batch_size"], shuffle=mode == "train",
                              modalities=self.config.get("modalities"),
                              missing_strategy=self.config.get("handle_missing_modalities",
                                                               self.config.get("missing_strategy", "zero_fill")),
                              target_size=tuple(self.config.get("target_size", (128, 128, 128))),
                              is_training=mode == "train", data_type=self.config.get("data_type", "BPH"),
                              rank=self.rank, world_size=self.world_size)

    def _broadcast_params(self):
        eng = self.model.engine()
        dist.broadcast(eng.flat_p, src=0)
        dist.broadcast(eng.flat_bn, src=0)
        eng.mark_dirty()

    # ---- the hot path ----
    def step(self, batch) -> float:
        loss = self.step_async(batch)
        return loss.item()

    def _grad_sync(self):
        eng = self.model.engine()
        if self._sync is None or self._sync.flat_g is not eng.flat_g:
            self._sync = GradSync(eng.flat_g, bucket_elems=self.config.get("dp_bucket_elems", 16 << 20),
                                  overlap=self.config.get("dp_overlap", True),
                                  min_bucket_elems=self.config.get("dp_min_bucket_elems", 1 << 20))
        return eng, self._sync

    def _clip_buffers(self):
        if self._clip_bufs is None:
            dev = self.model.engine().flat_g.device
            self._clip_bufs = (torch.empty(query("pcms_grad_clip_ws_doubles"), dtype=torch.float64, device=dev),
                               torch.empty(1, device=dev), torch.empty(1, device=dev))
        return self._clip_bufs

    def step_async(self, batch) -> torch.Tensor:
        """One training step; returns the loss as a device tensor (no host sync unless the
        AMP variant has to decide whether to skip the update)."""
        images = batch["image"].to(self.device, non_blocking=True)
        labels = batch["label"].to(self.device, non_blocking=True)
        if not self.model.training:  # (the engine follows UNet3D.training only)
            self.model.train()
        self.optimizer.zero_grad()
        if self.distributed:
            eng, sync = self._grad_sync()
            sync.reset()
            sync.broadcast_buffers(eng.flat_bn)
            eng.grad_ready = sync.ready   # buckets launch as the backward finishes each module
        try:
            outputs = self.model(images)
            loss = self.criterion(outputs, labels)
            root = self.scaler.scale(loss) if self.scaler is not None else loss
            # the backward's seed gradient held across steps (loss.backward() would fill a fresh
            # ones tensor on the device every step)
            seed = self._bw_seed
            if seed is None or seed.dtype != root.dtype or seed.device != root.device or seed.shape != root.shape:
                seed = self._bw_seed = torch.ones_like(root)
            torch.autograd.backward(root, grad_tensors=seed)
        except BaseException:
            if self.distributed:
                sync.reset()
            raise
        finally:
            if self.distributed:
                eng.grad_ready = None
        # sum over ranks -> mean: folded into the Adam pass (which writes the mean back)
        self.optimizer.grad_scale = sync.finish() if self.distributed else 1.0
        if self.scaler is not None:
            self.scaler._unscale(self.optimizer, max_norm=self.max_grad_norm or 0.0)
            self.last_grad_norm = self.scaler._norm
            self.scaler.step(self.optimizer)
            self.scaler.update()
        else:
            if self.max_grad_norm is not None:
                eng = self.model.engine()
                ws, norm, mul = self._clip_buffers()
                call("pcms_grad_clip", eng.flat_g, eng.flat_g.numel(), float(self.optimizer.grad_scale),
                     float(self.max_grad_norm), 0, ws, norm, mul)
                self.optimizer.grad_scale, self.optimizer.grad_mul = 1.0, mul
                self.last_grad_norm = norm
            self.optimizer.step()
        return loss.detach()

    def _prefetched(self, loader):
        """Yield batches whose H2D copy ran on a side stream while the previous step ran."""
        if self.device.type != "cuda":
            yield from loader
            return
        if self._copy_stream is None:
            self._copy_stream = torch.cuda.Stream(device=self.device)
        cs = self._copy_stream
        nxt = None
        for batch in loader:
            with torch.cuda.stream(cs):
                staged = {k: (v.pin_memory().to(self.device, non_blocking=True)
                              if torch.is_tensor(v) and v.device.type == "cpu" else v)
                          for k, v in batch.items()}
                ev = torch.cuda.Event()
                ev.record(cs)
            if nxt is not None:
                yield nxt
            main = torch.cuda.current_stream()
            main.wait_event(ev)
            for v in staged.values():
                if torch.is_tensor(v) and v.device.type == "cuda":
                    # allocated on the copy stream, used on the compute stream: keep the
                    # caching allocator from reusing the block before compute is done
                    v.record_stream(main)
            nxt = staged
        if nxt is not None:
            yield nxt

    def train_epoch(self):
        self.model.train()
        total, n = 0.0, 0
        for batch in self._prefetched(self.train_loader):
            total += self.step(batch)
            n += 1
        return total / max(n, 1)

    def _validate_sums(self):
        self.model.eval()
        total, n = 0.0, 0
        with torch.no_grad():
            for batch in self.val_loader:
                out = self.model(batch["image"].to(self.device))
                total += self.criterion(out, batch["label"].to(self.device)).item()
                n += 1
        return total, n

    def validate_epoch(self):
        """utils/trainer.py:201-234: the mean of the per-batch losses.  Under data
        parallelism each rank evaluates whole batches of the single-process batching
        (data.get_dataloader, ``is_training=False``: batches r, r + W, ...; no padding) and
        the (sum, count) pair is summed over ranks, so every rank gets the full-set value the
        single-process reference computes."""
        if self.val_loader is None:
            return None
        total, n = self._validate_sums()
        if self.distributed:
            t = torch.tensor([total, float(n)], dtype=torch.float64, device=self.model.engine().flat_p.device)
            dist.all_reduce(t)
            total, n = float(t[0]), int(t[1])
        return total / max(n, 1)

    def save_checkpoint(self, epoch, loss, is_best=False, best_loss=None, patience=None,
                        filename="latest_checkpoint.pth"):
        """utils/trainer.py:236-278 (same dict keys and file names; ``best_loss`` /
        ``patience`` are extra keys so a resumed ``train`` continues its early stopping).
        ``train`` writes ``latest_checkpoint.pth`` on improvement only, as the reference
        (:325-334), so that file always holds the best model and loss; the per-epoch resume
        state goes to ``filename="resume_checkpoint.pth"``."""
        if self.rank != 0:
            return
        ckpt = {"epoch": epoch, "model_state_dict": self.model.state_dict(),
                "optimizer_state_dict": self.optimizer.state_dict(),
                "scheduler_state_dict": self.scheduler.state_dict(), "loss": loss, "config": self.config}
        if best_loss is not None:
            ckpt["best_loss"], ckpt["patience"] = float(best_loss), int(patience or 0)
        if self.scaler is not None:
            ckpt["scaler_state_dict"] = self.scaler.state_dict()
        torch.save(ckpt, os.path.join(self.config["save_dir"], filename))
        if is_best:
            torch.save(self.model.state_dict(),
                       os.path.join(self.config["save_dir"], f"best_model_epoch_{epoch}.pth"))

    def load_checkpoint(self, path: str):
        """Resume from a ``save_checkpoint`` file (ours or the reference's: same keys, Adam
        state in torch.optim.Adam's format): model, optimizer and ReduceLROnPlateau state,
        and the early-stopping state (ours: ``best_loss`` / ``patience``; the reference's
        files: the saved ``loss`` as the best so far).  Returns ``(epoch, loss)``;
        ``train(start_epoch=epoch)`` continues from there."""
        ckpt = torch.load(path, map_location=self.device, weights_only=True)
        self.model.load_state_dict(ckpt["model_state_dict"])
        self.model.engine().mark_dirty()
        if "optimizer_state_dict" in ckpt:
            self.optimizer.load_state_dict(ckpt["optimizer_state_dict"])
        if "scheduler_state_dict" in ckpt:
            self.scheduler.load_state_dict(ckpt["scheduler_state_dict"])
        if self.scaler is not None and "scaler_state_dict" in ckpt:
            self.scaler.load_state_dict(ckpt["scaler_state_dict"])
        loss = ckpt.get("loss")
        best = ckpt.get("best_loss", loss if loss is not None else float("inf"))
        self._resume = (float(best), int(ckpt.get("patience", 0)))
        return int(ckpt.get("epoch", 0)), loss

    def _mean_over_ranks(self, v):
        """The epoch loss every rank acts on: the mean over ranks (so ReduceLROnPlateau and
        early stopping take the same decisions everywhere and no rank leaves the loop alone)."""
        if v is None or not self.distributed:
            return v
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.model.engine().flat_p.device)
        dist.all_reduce(t)
        return float(t) / self.world_size

    def train(self, start_epoch: int = 0, best_loss: Optional[float] = None):
        """Epoch loop with ReduceLROnPlateau and early stopping at patience 20 (:280-345).
        ``best_loss`` defaults to the value a loaded checkpoint carried (else inf)."""
        best, patience = self._resume
        if best_loss is not None:
            best, patience = float(best_loss), 0
        for epoch in range(start_epoch, self.config["num_epochs"]):
            for ld in (self.train_loader, self.val_loader):
                sampler = getattr(ld, "sampler", None)
                if hasattr(sampler, "set_epoch"):
                    sampler.set_epoch(epoch)
            train_loss = self._mean_over_ranks(self.train_epoch())
            if self.distributed:  # validate with rank 0's running statistics everywhere
                dist.broadcast(self.model.engine().flat_bn, src=0)
            val_loss = self.validate_epoch()  # already the full-set value on every rank
            cur = val_loss if val_loss is not None else train_loss
            self.scheduler.step(cur)
            improved = cur < best
            if improved:
                best, patience = cur, 0
            else:
                patience += 1
            if self.config.get("save_dir"):
                if improved:  # the reference's latest_checkpoint.pth (best model) + best_model_epoch_{e}.pth
                    self.save_checkpoint(epoch + 1, cur, is_best=True, best_loss=best, patience=patience)
                # every epoch: the state a resumed train() continues from (this epoch, this patience)
                self.save_checkpoint(epoch + 1, cur, best_loss=best, patience=patience,
                                     filename="resume_checkpoint.pth")
            if patience >= 20:
                break
        self._resume = (best, patience)
        return best


class Trainer(BaseTrainer):
    """The ``Trainer`` that run.py:30 imports (absent from the reference); BaseTrainer + step()."""
