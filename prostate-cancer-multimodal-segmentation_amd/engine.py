"""U-Net execution engine: the forward / backward schedule of the reference model over the
HIP kernels of libpcms_hip.so.

Reference call graph reproduced (models/unet3d.py):
  inc -> down1..down4 (MaxPool3d(2) + DoubleConv) -> up1..up4 (ConvT + pad + cat[skip, up]
  + DoubleConv) -> outc                                   forward @247-296
and its autograd backward (aten convolution_backward / batch_norm_backward / ...).

Layout: activations NDHWC in ``dtype`` (bf16 default, fp32 parity build); parameters live
in ONE flat fp32 master buffer (the module's nn.Parameters are views into it, so
``state_dict()`` keys/shapes are the reference's), gradients in one flat fp32 buffer
(``param.grad`` views), BatchNorm running stats in one flat fp32 buffer.  Kernel weight
packs (bf16 / fp32, MFMA-friendly order) are rebuilt from the master when it changes.

The engine keeps the activations of the LAST training forward; ``backward`` must follow
that forward (checked).  Only device code runs: there is no CPU path.
"""
from __future__ import annotations

import contextlib
import math
import os
from typing import Dict, List, Optional, Tuple

import torch

from . import _lib
from ._lib import BF16, F32, F32X3, call, query
from .dp import module_grad_ranges

BN_EPS = 1e-5
BN_MOMENTUM = 0.1

_DT = {"bf16": (torch.bfloat16, BF16), "fp32": (torch.float32, F32)}


class ConvSpec:
    __slots__ = ("mod", "cin", "cout", "cin_store", "fwd", "dgrad", "code", "fwd16", "dgrad16", "old_stale",
                 "old_used")

    def __init__(self, mod, cin, cout, cin_store):
        self.mod, self.cin, self.cout, self.cin_store = mod, cin, cout, cin_store
        self.fwd = None
        self.dgrad = None
        # pcms_conv3_pack16 forms for the 16x16x32 big-box kernel (pcms_conv3_fwd16), set by
        # UNetEngine._alloc for the convs whose forward / dgrad run on it at the allocated shape
        self.fwd16 = None
        self.dgrad16 = None
        # fwd / dgrad (the general kernel's packs) not rewritten by the last fused Adam (it
        # writes only the pack16 forms of a conv whose every call at the allocated shape ran
        # on the 16x16x32 kernel); old_used: a call at this shape needed them
        self.old_stale = False
        self.old_used = False
        # conv-kernel dtype code: BF16, or for fp32 data F32 (bf16x6 arithmetic, fp32-grade)
        # / F32X3 (bf16x3, faster, ~10x the fp32 rounding error)
        self.code = None


class BNSpec:
    __slots__ = ("mod", "c", "scale", "shift", "mean", "invstd")

    def __init__(self, mod, c):
        self.mod, self.c = mod, c
        self.scale = self.shift = self.mean = self.invstd = None


class BlockSpec:
    """DoubleConv3D: conv0 -> bn0 -> relu -> conv1 -> bn1 -> relu (models/unet3d.py:27-40)."""

    def __init__(self, dc, cin_store):
        seq = dc.conv
        self.c0 = ConvSpec(seq[0], seq[0].in_channels, seq[0].out_channels, cin_store)
        self.b0 = BNSpec(seq[1], seq[1].num_features)
        self.c1 = ConvSpec(seq[3], seq[3].in_channels, seq[3].out_channels, seq[3].in_channels)
        self.b1 = BNSpec(seq[4], seq[4].num_features)
        self.cout = self.c1.cout


def _round8(c: int) -> int:
    return (c + 7) // 8 * 8


class UNetEngine:
    def __init__(self, model, device: torch.device, precision: str = "bf16"):
        if device.type != "cuda":
            raise RuntimeError("pcms_amd runs on a ROCm device only (no CPU path); move the model to 'cuda'")
        _lib.load()
        self.model = model
        self.device = device
        self.precision = precision
        self.tdtype, self.code = _DT[precision]
        self.esize = 2 if self.code == BF16 else 4
        self.ncls = model.n_classes
        self.nmod = model.n_modalities
        self.cp = _round8(self.nmod)
        if self.ncls > 4:
            raise ValueError("the fused output head supports n_classes <= 4")
        m = model
        self.enc = [BlockSpec(m.inc, self.cp)]
        for i in range(1, 5):
            dc = getattr(m, f"down{i}").maxpool_conv[1]
            self.enc.append(BlockSpec(dc, dc.conv[0].in_channels))
        self.ups = []
        self.dec = []
        for i in range(1, 5):
            up = getattr(m, f"up{i}")
            self.ups.append(up.up)
            self.dec.append(BlockSpec(up.conv, up.conv.conv[0].in_channels))
        self.convs: List[ConvSpec] = []
        self.bns: List[BNSpec] = []
        for b in self.enc + self.dec:
            self.convs += [b.c0, b.c1]
            self.bns += [b.b0, b.b1]
        for cs in self.convs:
            cs.code = self.code
        self.convt_packs: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}
        # bf16 build: the stem runs on dedicated tap-packed kernels (HBM-bound)
        self.stem_fast = self.code == BF16 and self.cp == 8
        self.stem_sup = 0  # pcms_stem_supported bits for the allocated shape (set by _alloc)
        # PCMS_STEM_DENSE: the K-dense stem forward (9 tap rows of 3 kw x 5 channels) when the
        # weight has <= 5 input channels; 0 selects the 14-tap-pair kernel (A/B)
        self.stem_dense = 16 if self.nmod <= 5 else 0
        # a DoubleConv's first BatchNorm + ReLU applied inside its second conv's staging (forward:
        # pcms_conv3_fwd_bnin, weight gradient: pcms_conv3_wgrad_bnin) instead of a y1 -> a1 HBM
        # pass, on the layers both kernels run (levels 0-1, bf16); bit-identical to the unfused
        # pair (same arithmetic and rounding).  False: the a1 pass (A/B)
        self.fuse_bnin = True
        self._bnin_cache = {}
        # the level-0/1 convs (forward and dgrad) on the 16x16x32 big-box kernel
        # (pcms_conv3_fwd16, pack16 weights rebuilt with the other packs); PCMS_B16=0 keeps the
        # 32x32x16 big-box kernel (A/B)
        self.use_b16 = os.environ.get("PCMS_B16", "1") != "0"
        self._p16 = None  # pcms_conv3_pack16 table for the allocated shape
        # the blocks whose training forward ran fused (id(BlockSpec)): the backward and the
        # checkpointed recompute follow the forward's decision, not the current settings
        self._fwd_bnin = set()
        self.stem_pack = None
        self._flat_ptrs = None
        self._packed_version = -1
        self._dirty = True
        self._packs_fresh = False  # the fused Adam wrote every conv / ConvT pack (not the stem's)
        self._stem_conv_stale = False  # the stem's general-kernel pack skipped by the fast path
        self._adam_plan = None
        self.bufs = None
        self.buf_key = None
        self.epoch = 0
        self.saved_epoch = -1
        # decoder activation checkpointing: the decoder blocks'
        # pre-BN conv outputs and first ReLU output (y1, a1, y2) are not kept per level; the
        # forward writes them into one shared level-0-sized set and the backward recomputes
        # them level by level with the forward's BatchNorm coefficients (no statistics pass,
        # running stats untouched).  Every reduction in the library sums in a fixed order (split-K
        # slabs, BN partial rows, weight-gradient partial rows), so the recomputed tensors are
        # bit-identical to the forward's and two identical steps give identical results.
        self.act_ckpt = False
        self.split_target = 512  # split-K conv launches (levels 2-4): workgroups aimed at
        self.wgrad_target = 256  # conv weight-gradient workgroups: one round of 1 WG per CU (fewer partial rows to reduce than 512)
        self.grad_ready = None   # callable(lo, hi) per finished module gradient (dp.GradSync.ready)
        self.kernel_timer = None  # dict name -> [(start, end) events] (bench.py roofline timing)
        self.wgrad_side_stream = False  # ablation: weight gradients on a side stream (measured 119.9 vs 121.6 vol/s: off)
        # levels >= this run their conv weight gradients on the side stream (the deep levels'
        # small latency-bound launches beside the dgrad chain; the big levels' persistent grids
        # straggle when they share the chip).  99: never
        self.wgrad_side_min_level = 99
        # the ConvTranspose weight + bias gradient (HBM-bound: it streams the up-path gradient,
        # 268 MB at level 0) on the side stream beside the same layer's ConvT dgrad (also
        # HBM-bound, reading the same tensor); joined before the next block's backward.  Its
        # partial rows then get their own workspace (ctws_w) instead of sharing ctws.
        self.convt_wgrad_side = False
        # the encoder's MaxPool3d backward + BN-backward reduction without rewriting the block
        # output's gradient (pcms_maxpool_bwd_bn_sums), the pooled part added again in that
        # BatchNorm's apply (pcms_maxpool_bn_apply): the same dy bits, one write + read of the
        # level's tensor fewer.  Measured +0.19 % per step (the per-cell apply streams at ~5.3 TB/s
        # where the per-voxel apply it replaces runs at ~6.2; profiles/r6_pool_bn_apply_fused_ab.txt):
        # off, i.e. pcms_maxpool_bwd_bn + pcms_bn_relu_bwd_finish
        self.pool_bn_apply_fused = False
        # ablation only (tests/tools/step_ab.py nopack): skip the input pack, so the stem reads
        # the previous step's packed input -- bounds what folding pack_input into the stem
        # kernels could save; never set in the product (the forward is wrong with it)
        self.ablate_skip_pack_input = False
        self._side_stream = None
        self._side_used = False
        # eval mode: every BatchNorm folded into the conv before it (pcms_bn_fold) and the ReLU
        # applied in the conv epilogue (PCMS_CONV_RELU): conv -> BN -> ReLU is one pass
        # (models/unet3d.py:298-344 predict / inference).  False: the unfolded eval path.
        self.fold_bn_eval = True
        self._eval = None      # {conv index: (fwd pack, folded bias)}, "stem": stem pack
        self._eval_key = None
        self._bn_epoch = 0     # training forwards so far (each moves the running statistics)
        # weight generation: bumped by every change of the master weights the storage version
        # counter does not see (the fused Adam writes flat_p through the C-ABI), by
        # re-flattening and by a change of conv arithmetic; part of the eval-pack key
        self._wgen = 0
        self._store_ranges = None  # (stem_sup, fill plan) of _store_plan
        self._gstore = False       # this backward writes conv weight gradients (PCMS_GRAD_STORE)
        self._flatten()
        for bn in self.bns:
            c = bn.c
            bn.scale, bn.shift, bn.mean, bn.invstd = (torch.empty(c, device=device) for _ in range(4))

    def set_fp32_conv_mode(self, mode: str, convs=None):
        """fp32 build: the arithmetic of the 3x3x3 convs (all, or the indices ``convs`` of
        self.convs): "x6" (bf16x6, fp32-grade, the default) or "x3" (bf16x3)."""
        if self.code == BF16:
            raise ValueError("the bf16 build has one conv arithmetic")
        code = {"x6": F32, "x3": F32X3}[mode]
        for i, cs in enumerate(self.convs):
            if convs is None or i in convs:
                cs.code = code
                cs.fwd = cs.dgrad = None
        self._dirty = True
        self._wgen += 1
        self._adam_plan = None  # its table holds the old packs' pointers
        self._eval = None
        self.buf_key = None

    # ------------------------------------------------------------------ parameters
    def _flatten(self):
        """One flat fp32 master (params), grad and BN-buffer store; modules hold views."""
        params = list(self.model.parameters())
        total = sum(p.numel() for p in params)
        flat = torch.empty(total, dtype=torch.float32, device=self.device)
        gflat = torch.zeros(total, dtype=torch.float32, device=self.device)
        off = 0
        with torch.no_grad():
            for p in params:
                n = p.numel()
                flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = flat[off:off + n].view_as(p)
                if p.grad is not None:
                    gflat[off:off + n].copy_(p.grad.reshape(-1))
                p.grad = gflat[off:off + n].view_as(p)
                off += n
        bn_total = sum(2 * bn.c for bn in self.bns)
        bflat = torch.empty(bn_total, dtype=torch.float32, device=self.device)
        off = 0
        with torch.no_grad():
            for bn in self.bns:
                for name in ("running_mean", "running_var"):
                    t = getattr(bn.mod, name)
                    bflat[off:off + bn.c].copy_(t.reshape(-1))
                    t.data = bflat[off:off + bn.c]
                    off += bn.c
                nbt = bn.mod.num_batches_tracked
                if nbt.device != self.device:
                    nbt.data = nbt.data.to(self.device)
        self.params = params
        self.flat_p, self.flat_g, self.flat_bn = flat, gflat, bflat
        self._flat_ptrs = [p.data_ptr() for p in params]
        self._dirty = True
        self._wgen = getattr(self, "_wgen", 0) + 1
        self._adam_plan = None
        self._store_ranges = None  # offsets into the new flat buffer
        self._p16 = None           # weight pointers of the pack16 table
        self.grad_ranges = module_grad_ranges(self.model)
        # [lo, hi) of every parameter in the flat gradient (per-layer readiness for dp.GradSync)
        self.param_span = {}
        off = 0
        for p in params:
            self.param_span[id(p)] = (off, off + p.numel())
            off += p.numel()

    @contextlib.contextmanager
    def _timed(self, name: str):
        """HIP events around one library call on the current stream when ``kernel_timer`` (a
        dict name -> list) is set: bench.py times the stem kernels inside its timed steps."""
        t = self.kernel_timer
        if t is None:
            yield
            return
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        yield
        e1.record()
        t.setdefault(name, []).append((e0, e1))

    def _grads_done(self, *params):
        """The gradients of ``params`` (adjacent in the flat buffer) are final: report their
        flat range to the data-parallel hook (dp.GradSync) -- per layer, as each
        weight-gradient / BatchNorm-backward kernel is enqueued, in descending flat order
        (dp.readiness_groups lists the sequence), so the all-reduce buckets start while the
        backward still runs and only the last layers' bucket waits at the end.  With the
        weight gradients on the side stream the report is made from that stream after it has
        waited for the compute stream's queue, so a bucket's all-reduce is ordered after the
        kernels of both streams that wrote it, and the compute stream itself does not wait for
        the weight gradients (it joins them once per block: _block_bwd)."""
        if self.grad_ready is None:
            return
        spans = [self.param_span[id(p)] for p in params]
        lo, hi = min(a for a, _ in spans), max(b for _, b in spans)
        if self._side_used:
            side = self._side_stream
            side.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(side):
                self.grad_ready(lo, hi)
        else:
            self.grad_ready(lo, hi)

    # weight gradients run on a side stream beside the data-gradient chain (dgrad -> BN ->
    # dgrad ...): they only read activations and the dY buffer of their layer, which the main
    # stream does not overwrite before the next _join_side()
    def _side_at(self, lvl: int) -> bool:
        return self.wgrad_side_stream or lvl >= self.wgrad_side_min_level

    def _side(self, lvl: int, on: Optional[bool] = None):
        if not (self._side_at(lvl) if on is None else on):
            return contextlib.nullcontext()
        if self._side_stream is None:
            self._side_stream = torch.cuda.Stream(device=self.device)
        main = torch.cuda.current_stream(self.device)
        self._side_stream.wait_stream(main)
        self._side_used = True
        return torch.cuda.stream(self._side_stream)

    def _join_side(self):
        if self._side_used:
            torch.cuda.current_stream(self.device).wait_stream(self._side_stream)
            self._side_used = False

    def sync_params(self, full: bool = True, fresh_ok: bool = False) -> bool:
        """Re-flatten if a module op (``.to()``, ``.cuda()``, param reassignment) replaced
        storage, and make every ``param.grad`` a view of the flat gradient again.
        ``full=False`` (the calls inside one step after the forward's full check) skips the
        module walk that detects replaced Parameter objects.  ``fresh_ok`` (the backward):
        when EVERY gradient is None (``zero_grad(set_to_none=True)``, torch's default) the views
        are attached without zeroing and True is returned -- the backward then writes the
        gradient instead of accumulating into it (no 361 MB zero fill)."""
        if [p.data_ptr() for p in self.params] != self._flat_ptrs or (
                full and list(self.model.parameters()) != self.params):
            self._flatten()
            return False
        if all(p.grad is None for p in self.params):
            if not fresh_ok:
                return False  # stay None (torch semantics) until a backward attaches them
            off = 0
            for p in self.params:
                n = p.numel()
                p.grad = self.flat_g[off:off + n].view_as(p)
                off += n
            return True
        off = 0
        for p in self.params:
            n = p.numel()
            g = p.grad
            if g is None or g.data_ptr() != self.flat_g.data_ptr() + 4 * off:
                view = self.flat_g[off:off + n].view_as(p)
                with torch.no_grad():
                    if g is None:
                        view.zero_()
                    else:
                        view.copy_(g)
                p.grad = view
            off += n
        return False

    def _store_plan(self):
        """The flat-gradient ranges a fresh backward does NOT write with PCMS_GRAD_STORE (every
        parameter but the weights of the convs that go through pcms_conv3_wgrad): zeroed by one
        pcms_fill_ranges launch before such a backward.  Depends on the stem path (stem_sup)."""
        key = self.stem_sup
        if self._store_ranges is not None and self._store_ranges[0] == key:
            return self._store_ranges[1]
        base = self.flat_g.data_ptr()
        stored = []
        for i, cs in enumerate(self.convs):
            if i == 0 and self.stem_sup & 2:
                continue  # the stem's streaming kernel accumulates
            w = cs.mod.weight
            stored.append(((w.data_ptr() - self.flat_p.data_ptr()) // 4, w.numel()))
        ranges, pos = [], 0
        for off, n in sorted(stored):
            if off > pos:
                ranges.append([pos, off])
            pos = off + n
        if pos < self.flat_g.numel():
            ranges.append([pos, self.flat_g.numel()])
        plan = (torch.tensor(ranges, dtype=torch.int64, device=self.device), len(ranges),
                max(e - b for b, e in ranges))
        self._store_ranges = (key, plan)
        return plan

    def mark_dirty(self, packs_fresh: bool = False):
        """The master weights changed.  ``packs_fresh``: the fused Adam (adam_plan) already
        wrote the conv and ConvT packs from the new weights; only the stem's remain."""
        self._dirty = True
        self._wgen += 1
        self._packs_fresh = packs_fresh and self._packed_version == self.flat_p._version
        if self._packs_fresh and self._adam_plan is not None:
            for cs in self._adam_plan["old_skip"]:
                cs.old_stale = True

    def adam_plan(self):
        """Fused Adam + weight-pack plan (FlatAdam.step): device tables of the conv / ConvT
        weights whose packs the Adam kernels write (int64 rows, see include/pcms_hip.h
        pcms_adam_pack_conv3) and the [begin, end) ranges of every other parameter.  The bf16
        build writes bf16 packs; the fp32 build (``"x6"``: True) its bf16x6 packs, for the
        convs in bf16x6 mode (a conv switched to bf16x3 is repacked as before)."""
        if self._adam_plan is not None:
            return self._adam_plan
        x6 = self.code != BF16
        self._ensure_packs()
        base = self.flat_p.data_ptr()

        def offset(t):
            return (t.data_ptr() - base) // 4

        fused = []
        skipped = 0  # layers (besides the stem) whose packs the Adam kernels do not write
        conv_rows, tiles, old_skip = [], 0, []
        for i, cs in enumerate(self.convs):
            w = cs.mod.weight
            if i == 0:
                continue
            if cs.cin % 32 or cs.cout % 32 or offset(w) % 4 or (x6 and cs.code != F32):
                skipped += 1
                continue
            # bf16 build: the pack16 forms too; the general kernel's packs only where a call
            # at this shape used them (else marked stale, repacked on first use: _old_packs)
            f16 = cs.fwd16.data_ptr() if not x6 and cs.fwd16 is not None else 0
            d16 = cs.dgrad16.data_ptr() if not x6 and cs.dgrad16 is not None else 0
            skip = bool(f16 and d16) and not cs.old_used
            conv_rows.append([offset(w), cs.cout, cs.cin, 0 if skip else cs.fwd.data_ptr(),
                              0 if skip else cs.dgrad.data_ptr(), tiles, f16, d16])
            if skip:
                old_skip.append(cs)
            tiles += (cs.cout // 32) * (cs.cin // (16 if x6 else 32))
            fused.append((offset(w), w.numel()))
        ct_rows, ct_tiles = [], 0
        for i, up in enumerate(self.ups):
            w = up.weight
            cin, cout = up.in_channels, up.out_channels
            if cin % 32 or cout % 32 or offset(w) % 4:
                skipped += 1
                continue
            f, d = self.convt_packs[i]
            ct_rows.append([offset(w), cin, cout, f.data_ptr(), d.data_ptr(), ct_tiles, 0, 0])
            ct_tiles += (cin // 32) * (cout // 32)
            fused.append((offset(w), w.numel()))
        ranges, pos = [], 0
        for off, n in sorted(fused):
            if off > pos:
                ranges.append([pos, off])
            pos = off + n
        if pos < self.flat_p.numel():
            ranges.append([pos, self.flat_p.numel()])
        dev = self.device

        def tab(rows):
            return torch.tensor(rows if rows else [[0] * 8], dtype=torch.int64, device=dev)
        self._adam_plan = {
            "conv": tab(conv_rows), "nconv": len(conv_rows), "conv_tiles": tiles,
            "convt": tab(ct_rows), "nconvt": len(ct_rows), "convt_tiles": ct_tiles,
            "ranges": torch.tensor(ranges if ranges else [[0, 0]], dtype=torch.int64, device=dev),
            "nranges": len(ranges), "max_len": max([e - b for b, e in ranges], default=0),
            # every conv / ConvT pack but the stem's comes out of the Adam pass (else the step
            # must not mark the packs fresh: a skipped layer would train on stale packs)
            "complete": skipped == 0,
            "x6": x6,
            "old_skip": old_skip,  # convs whose general-kernel packs this plan does not write
            "p16": not x6,         # the pack16 forms come out of the Adam pass
        }
        return self._adam_plan

    def _ensure_packs(self):
        v = self.flat_p._version
        if not self._dirty and v == self._packed_version:
            return
        if self._packs_fresh and v == self._packed_version:
            # the fused Adam rewrote every conv / ConvT pack: only the stem's are left.  With
            # the direct stem kernels its general-kernel pack is needed only by a shape they do
            # not run (packed on first use there: _conv)
            cs = self.convs[0]
            if self.stem_fast:
                call("pcms_stem_pack", cs.mod.weight, self.stem_pack, self.nmod)
                self._stem_conv_stale = True
            elif cs.dgrad is None:
                call("pcms_conv3_pack", cs.code, cs.mod.weight, cs.fwd, cs.cout, cs.cin, 0)
            else:
                call("pcms_conv3_pack2", cs.code, cs.mod.weight, cs.fwd, cs.dgrad, cs.cout, cs.cin)
            self._dirty = False
            self._packs_fresh = False
            if self._adam_plan is None or not self._adam_plan["p16"]:
                self._pack16()
            return
        for i, cs in enumerate(self.convs):
            w = cs.mod.weight
            if cs.fwd is None:
                cs.fwd = torch.empty(query("pcms_conv3_pack_elems", cs.code, cs.cout, cs.cin), dtype=self.tdtype,
                                     device=self.device)
                if i != 0:  # the stem's input needs no gradient -> no dgrad pack
                    cs.dgrad = torch.empty(query("pcms_conv3_pack_elems", cs.code, cs.cin, cs.cout),
                                           dtype=self.tdtype, device=self.device)
            if cs.dgrad is not None:
                call("pcms_conv3_pack2", cs.code, w, cs.fwd, cs.dgrad, cs.cout, cs.cin)
            else:
                call("pcms_conv3_pack", cs.code, w, cs.fwd, cs.cout, cs.cin, 0)
        if self.stem_fast:
            if self.stem_pack is None:
                self.stem_pack = torch.empty(query("pcms_stem_pack_elems"), dtype=self.tdtype, device=self.device)
            call("pcms_stem_pack", self.convs[0].mod.weight, self.stem_pack, self.nmod)
        for i, up in enumerate(self.ups):
            cin, cout = up.in_channels, up.out_channels
            if i not in self.convt_packs:
                n = query("pcms_convt_pack_elems", self.code, cin, cout)
                self.convt_packs[i] = (torch.empty(n, dtype=self.tdtype, device=self.device),
                                       torch.empty(n, dtype=self.tdtype, device=self.device))
            f, d = self.convt_packs[i]
            call("pcms_convt_pack", self.code, up.weight, f, cin, cout, 0)
            call("pcms_convt_pack", self.code, up.weight, d, cin, cout, 1)
        for cs in self.convs:
            cs.old_stale = False
        self._packed_version = self.flat_p._version
        self._dirty = False
        self._packs_fresh = False
        self._stem_conv_stale = False
        self._pack16()

    def _pack16(self):
        """The pack16 forms of the convs running on the 16x16x32 big-box kernel at the allocated
        shape: one batched pcms_conv3_pack16 launch from the fp32 master (its table is rebuilt
        when the buffers or the flat parameters move)."""
        if self._p16 is None:
            rows, tiles = [], 0
            for cs in self.convs:
                if cs.fwd16 is None and cs.dgrad16 is None:
                    continue
                rows.append([cs.mod.weight.data_ptr(), cs.cout, cs.cin, 0 if cs.fwd16 is None else cs.fwd16.data_ptr(),
                             0 if cs.dgrad16 is None else cs.dgrad16.data_ptr(), tiles, 0, 0])
                tiles += (cs.cout // 32) * (cs.cin // 32)
            self._p16 = (torch.tensor(rows if rows else [[0] * 8], dtype=torch.int64, device=self.device), len(rows),
                         tiles)
        tab, n, tiles = self._p16
        if n:
            call("pcms_conv3_pack16", tab, n, tiles)

    def _old_packs(self, cs: ConvSpec):
        """The general kernel's packs of ``cs`` before a call that reads them: rebuilt from the
        master when the fused Adam skipped them, and the Adam plan redone so that it writes
        them from the next step on."""
        if cs.old_stale:
            call("pcms_conv3_pack2", cs.code, cs.mod.weight, cs.fwd, cs.dgrad, cs.cout, cs.cin)
            cs.old_stale = False
        if not cs.old_used:
            cs.old_used = True
            self._adam_plan = None

    def _stem_conv_pack(self):
        """The stem conv's general-kernel weight pack, when the fast path skipped it."""
        if self._stem_conv_stale:
            cs = self.convs[0]
            if cs.dgrad is None:
                call("pcms_conv3_pack", cs.code, cs.mod.weight, cs.fwd, cs.cout, cs.cin, 0)
            else:
                call("pcms_conv3_pack2", cs.code, cs.mod.weight, cs.fwd, cs.dgrad, cs.cout, cs.cin)
            self._stem_conv_stale = False

    def _ensure_eval_packs(self):
        """Folded eval weights: w' = w * gamma / sqrt(rvar + eps), b' = b * sc + beta - rmean * sc
        per conv (pcms_bn_fold, then the forward pack of w'); rebuilt when the parameters or
        the running statistics changed."""
        self._ensure_packs()
        key = (self._wgen, self.flat_p._version, self.flat_bn._version, self._bn_epoch)
        if self._eval is not None and self._eval_key == key:
            return
        if self._eval is None:
            self._eval = {}
            big = max(cs.cout * cs.cin * 27 for cs in self.convs)
            self._eval_tmp = torch.empty(big, dtype=torch.float32, device=self.device)
        tmp = self._eval_tmp
        for i, (cs, bn) in enumerate(zip(self.convs, self.bns)):
            if i not in self._eval:
                self._eval[i] = (torch.empty(query("pcms_conv3_pack_elems", cs.code, cs.cout, cs.cin),
                                             dtype=self.tdtype, device=self.device),
                                 torch.empty(cs.cout, dtype=torch.float32, device=self.device))
            pack, bias = self._eval[i]
            m = bn.mod
            call("pcms_bn_fold", cs.mod.weight, cs.mod.bias, m.weight, m.bias, m.running_mean, m.running_var,
                 BN_EPS, cs.cout, cs.cin * 27, tmp, bias)
            call("pcms_conv3_pack", cs.code, tmp, pack, cs.cout, cs.cin, 0)
            if i == 0 and self.stem_fast:
                if "stem" not in self._eval:
                    self._eval["stem"] = torch.empty(query("pcms_stem_pack_elems"), dtype=self.tdtype,
                                                     device=self.device)
                call("pcms_stem_pack", tmp, self._eval["stem"], self.nmod)
        self._eval_key = key

    def _conv_eval(self, i: int, x0, c0, x1, c1, a, N, S):
        """a = relu(conv'(x) + b'): the folded eval conv of self.convs[i] (no statistics)."""
        cs = self.convs[i]
        pack, bias = self._eval[i]
        RELU = 2  # PCMS_CONV_RELU
        splits = self._splits(N, S, c0 + c1, cs.cout, cs.code)
        if i == 0 and self.stem_sup & 1:
            call("pcms_stem_fwd", x0, self._eval["stem"], bias, a, None, N, S[0], S[1], S[2], RELU | self.stem_dense)
        elif splits == 1:
            call("pcms_conv3_fwd", cs.code, x0, c0, x1, c1, pack, bias, a, None, cs.cout, None, None, RELU,
                 N, S[0], S[1], S[2], cs.cout, 1)
        else:
            acc = self.bufs["yacc"]
            call("pcms_conv3_fwd", cs.code, x0, c0, x1, c1, pack, bias, a, None, cs.cout, acc, None, 0,
                 N, S[0], S[1], S[2], cs.cout, splits)
            call("pcms_split_epilogue", self.code, acc, query("pcms_conv3_splits", cs.code, c0 + c1, splits),
                 bias, a, None, cs.cout, None, cs.cout, N * S[0] * S[1] * S[2], RELU)

    # ------------------------------------------------------------------ buffers
    def _levels(self, D, H, W):
        s = [(D, H, W)]
        for _ in range(4):
            d, h, w = s[-1]
            s.append((d // 2, h // 2, w // 2))
        return s

    def _alloc(self, N, D, H, W):
        # the workspaces below are sized for the current split / weight-gradient workgroup
        # targets: a changed target re-lays them out (a larger one would otherwise overrun them)
        key = (N, D, H, W, self.act_ckpt, self.wgrad_side_stream, self.wgrad_side_min_level, self.wgrad_target,
               self.split_target, self.convt_wgrad_side)
        if self.buf_key == key:
            return
        self.bufs = None
        S = self._levels(D, H, W)
        if min(S[4]) < 1:
            raise ValueError(f"spatial size {(D, H, W)} is too small for 4 poolings")
        nv = [N * d * h * w for (d, h, w) in S]
        C = [64 * (1 << l) for l in range(5)]
        T = self.tdtype
        dev = self.device

        def act(l, c):
            return torch.empty(nv[l] * c, dtype=T, device=dev)

        b: Dict[str, object] = {"S": S, "nv": nv, "C": C}
        b["xin"] = act(0, self.cp)
        for l in range(5):
            if l > 0:
                b[f"pool{l}"] = act(l, C[l - 1])
            for k in ("y1", "a1", "y2", "x"):
                b[f"e{l}_{k}"] = act(l, C[l])
        for l in range(4):
            for k in (("u", "a2") if self.act_ckpt else ("u", "y1", "a1", "y2", "a2")):
                # the last decoder block's ReLU output is never stored: the head applies that
                # BatchNorm + ReLU itself (pcms_head_bn_fwd / _bwd)
                b[f"d{l}_{k}"] = act(l, C[l]) if (l, k) != (0, "a2") else None
        if self.act_ckpt:  # shared decoder set (level 0 is the largest: bytes per level ~ 4^-l)
            for k in ("y1", "a1", "y2"):
                b[f"ck_{k}"] = act(0, C[0])
        # gradient buffers
        for l in range(5):
            b[f"gx{l}"] = act(l, C[l])      # grad of encoder output x_l (skip + path)
            b[f"gA{l}"] = act(l, C[l])      # grad of a1 / block outputs (scratch)
            b[f"gY{l}"] = act(l, C[l])      # grad of pre-BN conv outputs (scratch)
            # second one while the side stream may still read gY; else an alias
            b[f"gZ{l}"] = act(l, C[l]) if self._side_at(l) else b[f"gY{l}"]
            b[f"gU{l}"] = act(l, C[l])      # grad of up output / pooled input (scratch)
        # workspaces
        rows_f = max(max(query("pcms_conv3_mblocks", N, *S[l]) for l in range(5)),
                     query("pcms_stem_fwd_rows", N, *S[0]))
        for blk, l in [(bk, i) for i, bk in enumerate(self.enc)] + [(bk, 3 - i) for i, bk in enumerate(self.dec)]:
            for cs, c1 in ((blk.c0, C[l] if blk in self.dec else 0), (blk.c1, 0)):
                rows_f = max(rows_f, query("pcms_conv3_fwd16_rows", N, *S[l], cs.cin_store - c1, c1, cs.cout))
        rows_s = max(query("pcms_split_epilogue_rows", nv[l]) for l in range(5))
        rows_b = max(query("pcms_bn_bwd_rows", self.code, C[l], nv[l]) for l in range(5))
        # BN partials [rows][C][2] + [rows] voxel counts
        # (also the fused head's BatchNorm partial rows [rows_h][64][2])
        rows_h = query("pcms_head_bn_bwd_rows", D * H * W, N)
        rows_b = max([rows_b] + [query("pcms_maxpool_bwd_bn_rows", self.code, N, *S[l], C[l]) for l in range(4)])
        b["stats"] = torch.empty(max(max(rows_f, rows_s, rows_b) * (1024 * 2 + 1), rows_h * 64 * 2),
                                 dtype=torch.float32, device=dev)
        b["coef"] = torch.empty(3 * 1024, dtype=torch.float32, device=dev)
        b["bnws"] = torch.empty(query("pcms_bn_ws_doubles", 1024), dtype=torch.float64, device=dev)
        # weight-gradient workspace: per-split partial rows of the largest conv (and the stem)
        ws = [query("pcms_stem_wgrad_ws_floats", N, *S[0], self.nmod)] if self.stem_fast else [1]
        for blk, l in [(bk, i) for i, bk in enumerate(self.enc)] + [(bk, 3 - i) for i, bk in enumerate(self.dec)]:
            for cs, c1 in ((blk.c0, C[l] if blk in self.dec else 0), (blk.c1, 0)):
                c0 = cs.cin_store - c1
                ws.append(query("pcms_conv3_wgrad_ws_floats", cs.code, N, *S[l], c0, c1, cs.cout,
                                self.wgrad_target))
        b["dwt"] = torch.empty(max(ws), dtype=torch.float32, device=dev)
        # split-K slabs [splits][nvox][Cout] for every conv (fwd and dgrad) that splits
        yacc = 1
        for blk, l in [(bk, i) for i, bk in enumerate(self.enc)] + [(bk, 3 - i) for i, bk in enumerate(self.dec)]:
            for cs, c1 in ((blk.c0, C[l] if blk in self.dec else 0), (blk.c1, 0)):
                # forward (sources as the block feeds them: the decoder's first conv reads the
                # skip and the upsampled halves), dgrad (the stem has none)
                dirs = [(cs.cin_store - c1, c1, cs.cout)] + ([(cs.cout, 0, cs.cin)] if cs is not self.convs[0] else [])
                for c0_, c1_, cout in dirs:
                    sp = self._splits(N, S[l], c0_ + c1_, cout, cs.code)
                    if sp > 1:
                        yacc = max(yacc, query("pcms_conv3_splits", cs.code, c0_ + c1_, sp) * nv[l] * cout)
                    if self.use_b16 and self.code == BF16:  # the level-3 16x16x32 split-K form
                        yacc = max(yacc, query("pcms_conv3_fwd16_split_ok", N, *S[l], c0_, c1_, cout) * nv[l] * cout)
        b["yacc"] = torch.empty(yacc, dtype=torch.float32, device=dev)
        # partial rows of the head / ConvT-bias gradient reductions (summed in a fixed order)
        red = [query("pcms_head_bwd_ws_floats", D * H * W, N, self.ncls)]
        for i, up in enumerate(self.ups):
            l = 3 - i
            red.append(query("pcms_convt_wgrad_bias_ws_floats", self.code, N, *S[l + 1], up.in_channels,
                             up.out_channels, 512))
        b["redws"] = torch.empty(max(red), dtype=torch.float32, device=dev)
        # dedicated stem kernels where they support the shape (else the general conv kernels)
        self.stem_sup = query("pcms_stem_supported", N, D, H, W) if self.stem_fast else 0
        ctws = [query("pcms_convt_wgrad_ws_floats", N, *S[4 - i], up.in_channels, up.out_channels, 512)
                for i, up in enumerate(self.ups)]
        if self.convt_wgrad_side:  # the weight gradient's rows apart: the dgrad runs beside it
            b["ctws_w"] = torch.empty(max(ctws), dtype=torch.float32, device=dev)
            ctws = []
        # the ConvT dgrad's K slabs share it (the weight gradient has reduced it by then)
        ctws += [query("pcms_convt_dgrad_ws_floats", N, *S[4 - i], up.in_channels, up.out_channels)
                 for i, up in enumerate(self.ups)]
        # and the forward's K slabs (free in the forward pass)
        ctws += [query("pcms_convt_fwd_ws_floats", N, *S[4 - i], up.in_channels, up.out_channels)
                 for i, up in enumerate(self.ups)]
        b["ctws"] = torch.empty(max(ctws), dtype=torch.float32, device=dev)
        # the 16x16x32 big-box kernel: forward (sources as the block feeds them) and dgrad
        for cs in self.convs:
            cs.fwd16 = cs.dgrad16 = None
        if self.use_b16 and self.code == BF16:
            for blk, l in [(bk, i) for i, bk in enumerate(self.enc)] + [(bk, 3 - i) for i, bk in enumerate(self.dec)]:
                for cs, c1 in ((blk.c0, C[l] if blk in self.dec else 0), (blk.c1, 0)):
                    if cs is self.convs[0]:
                        continue  # the stem runs on its own kernels
                    c0 = cs.cin_store - c1
                    if query("pcms_conv3_big16_ok", N, *S[l], c0, c1, cs.cout) or \
                            query("pcms_conv3_fwd16_split_ok", N, *S[l], c0, c1, cs.cout):
                        cs.fwd16 = torch.empty(query("pcms_conv3_pack16_elems", cs.cout, cs.cin), dtype=T, device=dev)
                    if query("pcms_conv3_big16_ok", N, *S[l], cs.cout, 0, cs.cin) or \
                            query("pcms_conv3_fwd16_split_ok", N, *S[l], cs.cout, 0, cs.cin):
                        cs.dgrad16 = torch.empty(query("pcms_conv3_pack16_elems", cs.cin, cs.cout), dtype=T, device=dev)
        for cs in self.convs:
            cs.old_used = False
        self._p16 = None
        self._dirty = True  # build the new pack16 forms before the next conv
        self._packs_fresh = False  # (those of the last fused Adam went to the old buffers)
        self._adam_plan = None
        self.bufs = b
        self.buf_key = key

    # ------------------------------------------------------------------ primitives
    def _splits(self, N, S, cin, cout, code):
        mb = query("pcms_conv3_mblocks", N, *S)
        wgs = mb * (cout // 64)
        nch = -(-cin // query("pcms_conv3_chunk", code))
        if wgs >= 192 or nch == 1 or wgs == 0:
            return 1
        return max(1, min(nch, -(-self.split_target // wgs)))

    def _bnin(self, blk: BlockSpec, N, S) -> bool:
        """The block's first BN + ReLU fused into its second conv (forward and weight gradient)?"""
        if not self.fuse_bnin or self.code != BF16:
            return False
        key = (id(blk), N, tuple(S), self.wgrad_target, self.split_target)
        if key not in self._bnin_cache:
            # only where the unfused conv runs unsplit (the same big-box kernel, so the fused
            # step stays bit-identical to the unfused one)
            self._bnin_cache[key] = bool(query("pcms_conv3_bnin_ok", N, *S, blk.c1.cin, blk.c1.cout,
                                               self.wgrad_target)) and \
                self._splits(N, S, blk.c1.cin, blk.c1.cout, self.code) == 1
        return self._bnin_cache[key]

    def _conv(self, cs: ConvSpec, x0, c0, x1, c1, y, N, S, stats: bool, training: bool, bn: BNSpec,
              recompute: bool = False, bnin: Optional[BNSpec] = None):
        """y = conv(x) + b; then BN statistics (train) or eval coefficients.  ``recompute``:
        the conv alone (checkpointed decoder: the forward's BN coefficients are reused).
        ``bnin``: the input is the pre-BN y1 of that BatchNorm; conv(relu(bn(x)))."""
        b = self.bufs
        nvox = N * S[0] * S[1] * S[2]
        splits = self._splits(N, S, c0 + c1, cs.cout, cs.code)
        st = b["stats"] if training and not recompute else None
        if cs is self.convs[0] and not self.stem_sup & 1:
            self._stem_conv_pack()
        if bnin is not None and cs.fwd16 is not None:
            call("pcms_conv3_fwd16", x0, c0, None, 0, bnin.scale, bnin.shift, cs.fwd16, cs.mod.bias, y, None, cs.cout,
                 st, 0, N, *S, cs.cout)
            rows = query("pcms_conv3_fwd16_rows", N, *S, c0, 0, cs.cout)
        elif bnin is not None:
            self._old_packs(cs)
            call("pcms_conv3_fwd_bnin", cs.code, x0, c0, bnin.scale, bnin.shift, cs.fwd, cs.mod.bias, y, st, N,
                 *S, cs.cout)
            rows = query("pcms_conv3_fwd_rows", cs.code, N, *S, c0, 0, cs.cout)
        elif cs is self.convs[0] and self.stem_sup & 1:
            with self._timed("stem_fwd"):
                call("pcms_stem_fwd", x0, self.stem_pack, cs.mod.bias, y, st, N, S[0], S[1], S[2], self.stem_dense)
            rows = query("pcms_stem_fwd_rows", N, *S)
        elif splits == 1 and cs.fwd16 is not None and query("pcms_conv3_big16_ok", N, *S, c0, c1, cs.cout):
            call("pcms_conv3_fwd16", x0, c0, x1, c1, None, None, cs.fwd16, cs.mod.bias, y, None, cs.cout, st, 0,
                 N, S[0], S[1], S[2], cs.cout)
            rows = query("pcms_conv3_fwd16_rows", N, *S, c0, c1, cs.cout)
        elif cs.fwd16 is not None and (sp16 := query("pcms_conv3_fwd16_split_ok", N, *S, c0, c1, cs.cout)):
            acc = b["yacc"]
            if sp16 * nvox * cs.cout > acc.numel():
                raise RuntimeError("split-K workspace smaller than the 16x16x32 split form needs")
            call("pcms_conv3_fwd16_split", x0, c0, x1, c1, cs.fwd16, acc, N, *S, cs.cout, sp16)
            call("pcms_split_epilogue", self.code, acc, sp16, cs.mod.bias, y, None, cs.cout, st, cs.cout, nvox, 0)
            rows = query("pcms_split_epilogue_rows", nvox)
        elif splits == 1:
            self._old_packs(cs)
            call("pcms_conv3_fwd", cs.code, x0, c0, x1, c1, cs.fwd, cs.mod.bias, y, None, cs.cout,
                 None, st, 0, N, S[0], S[1], S[2], cs.cout, 1)
            rows = query("pcms_conv3_fwd_rows", cs.code, N, *S, c0, c1, cs.cout)
        else:
            acc = b["yacc"]
            self._old_packs(cs)
            call("pcms_conv3_fwd", cs.code, x0, c0, x1, c1, cs.fwd, cs.mod.bias, y, None, cs.cout,
                 acc, None, 0, N, S[0], S[1], S[2], cs.cout, splits)
            call("pcms_split_epilogue", self.code, acc, query("pcms_conv3_splits", cs.code, c0 + c1, splits),
                 cs.mod.bias, y, None, cs.cout, st, cs.cout, nvox, 0)
            rows = query("pcms_split_epilogue_rows", nvox)
        if recompute:
            return
        m = bn.mod
        if training:
            if nvox <= 1:
                raise ValueError(f"Expected more than 1 value per channel when training, got input size "
                                 f"torch.Size([{N}, {bn.c}, {S[0]}, {S[1]}, {S[2]}])")
            call("pcms_bn_finalize", st, rows, bn.c, float(nvox), m.weight, m.bias, m.running_mean,
                 m.running_var, m.num_batches_tracked, BN_MOMENTUM, BN_EPS, bn.scale, bn.shift, bn.mean,
                 bn.invstd, b["bnws"])
        else:
            call("pcms_bn_eval_coeffs", m.weight, m.bias, m.running_mean, m.running_var, BN_EPS, bn.c,
                 bn.scale, bn.shift)

    def _block_fwd(self, blk: BlockSpec, x0, c0, x1, c1, out: Dict[str, torch.Tensor], N, S, training,
                   recompute: bool = False, pool_out=None):
        """conv -> BN -> ReLU -> conv -> BN -> ReLU.  ``recompute`` (checkpointed decoder
        backward): y1, a1, y2 again from the same inputs with the forward's BN scale/shift; no
        statistics, no running-stat update, a2 not rewritten.  ``out["a2"] is None``: the
        second BN + ReLU is left to the consumer (the head: pcms_head_bn_fwd).  ``pool_out``
        (encoder blocks 0-3): the output is max-pooled into it in the same pass (the next
        Down3D's MaxPool3d, pcms_bn_relu_pool)."""
        nvox = N * S[0] * S[1] * S[2]
        if not training and self.fold_bn_eval:
            # eval: BN folded, ReLU in the epilogue; the last decoder block's output goes to its
            # y2 buffer, which the plain head then reads (forward(): self._eval_folded)
            i0 = self.convs.index(blk.c0)
            a2 = out["a2"] if out["a2"] is not None else out["y2"]
            self._conv_eval(i0, x0, c0, x1, c1, out["a1"], N, S)
            self._conv_eval(i0 + 1, out["a1"], blk.c0.cout, None, 0, a2, N, S)
            if pool_out is not None:
                call("pcms_maxpool_fwd", self.code, a2, pool_out, N, *S, blk.c1.cout)
            return
        self._conv(blk.c0, x0, c0, x1, c1, out["y1"], N, S, True, training, blk.b0, recompute)
        if recompute:
            bnin = id(blk) in self._fwd_bnin
        else:
            bnin = self._bnin(blk, N, S)
            if training:
                (self._fwd_bnin.add if bnin else self._fwd_bnin.discard)(id(blk))
        if bnin:  # a1 is never stored: the second conv applies BN0 + ReLU itself
            self._conv(blk.c1, out["y1"], blk.c0.cout, None, 0, out["y2"], N, S, True, training, blk.b1, recompute,
                       bnin=blk.b0)
        else:
            call("pcms_bn_relu", self.code, out["y1"], out["a1"], blk.b0.scale, blk.b0.shift, blk.c0.cout, nvox)
            self._conv(blk.c1, out["a1"], blk.c0.cout, None, 0, out["y2"], N, S, True, training, blk.b1, recompute)
        if recompute or out["a2"] is None:
            return
        if pool_out is not None:
            call("pcms_bn_relu_pool", self.code, out["y2"], out["a2"], pool_out, blk.b1.scale, blk.b1.shift, N, *S,
                 blk.c1.cout)
        else:
            call("pcms_bn_relu", self.code, out["y2"], out["a2"], blk.b1.scale, blk.b1.shift, blk.c1.cout, nvox)

    def _dec_acts(self, l: int) -> Dict[str, torch.Tensor]:
        b = self.bufs
        if not self.buf_key[4]:  # the mode the buffers were laid out for
            return {k: b[f"d{l}_{k}"] for k in ("y1", "a1", "y2", "a2")}
        n = b["nv"][l] * b["C"][l]
        return {"y1": b["ck_y1"][:n], "a1": b["ck_a1"][:n], "y2": b["ck_y2"][:n], "a2": b[f"d{l}_a2"]}

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, training: bool, act: int = 0, threshold: float = 0.5) -> torch.Tensor:
        """The network on ``x`` (N, n_modalities, D, H, W).  ``act``: 0 logits, 1 sigmoid
        probabilities (predict), 2 ``sigmoid > threshold`` masks (inference), all produced
        by the head kernel."""
        if x.dim() != 5 or x.shape[1] != self.nmod:
            raise ValueError(f"expected input (N, {self.nmod}, D, H, W), got {tuple(x.shape)}")
        if x.device != self.device:
            raise ValueError(f"input on {x.device}, model on {self.device}")
        x = x.contiguous()
        if x.dtype != torch.float32:
            x = x.float()
        N, _, D, H, W = x.shape
        # buffers first: a (re)allocation decides which convs run on the 16x16x32 kernel and
        # marks the packs dirty, so their pack16 forms are built by the _ensure_packs below
        self._alloc(N, D, H, W)
        self._ensure_packs()
        folded = not training and self.fold_bn_eval
        if folded:
            self._ensure_eval_packs()
        else:
            self._bn_epoch += training
        b = self.bufs
        S, C = b["S"], b["C"]
        if not self.ablate_skip_pack_input:
            call("pcms_pack_input", self.code, x, b["xin"], N, self.nmod, D * H * W, self.cp)
        # encoder
        inp, cin = b["xin"], self.cp
        for l in range(5):
            if l > 0:  # pool{l} was written by the previous block's fused BN + ReLU + MaxPool pass
                inp, cin = b[f"pool{l}"], C[l - 1]
            out = {"y1": b[f"e{l}_y1"], "a1": b[f"e{l}_a1"], "y2": b[f"e{l}_y2"], "a2": b[f"e{l}_x"]}
            self._block_fwd(self.enc[l], inp, cin, None, 0, out, N, S[l], training,
                            pool_out=b[f"pool{l + 1}"] if l < 4 else None)
        # decoder
        h = b["e4_x"]
        for i in range(4):
            l = 3 - i
            up = self.ups[i]
            fpack, _ = self.convt_packs[i]
            call("pcms_convt_fwd_ws", self.code, h, fpack, up.bias, b[f"d{l}_u"], b["ctws"], N, *S[l + 1],
                 up.in_channels, up.out_channels, *S[l])
            self._block_fwd(self.dec[i], b[f"e{l}_x"], C[l], b[f"d{l}_u"], C[l], self._dec_acts(l), N, S[l],
                            training)
            h = b[f"d{l}_a2"]
        # head = the last decoder block's BN + ReLU + outc 1x1x1 conv in one pass over its y2
        logits = torch.empty((N, self.ncls, D, H, W), dtype=torch.float32, device=self.device)
        oc = self.model.outc
        bn = self.dec[3].b1
        if folded:  # the y2 buffer holds the folded conv's ReLU output
            call("pcms_head_fwd", self.code, self._dec_acts(0)["y2"], oc.weight, oc.bias, logits, D * H * W, N,
                 self.ncls, int(act), float(threshold))
        else:
            call("pcms_head_bn_fwd", self.code, self._dec_acts(0)["y2"], bn.scale, bn.shift, oc.weight, oc.bias,
                 logits, D * H * W, N, self.ncls, int(act), float(threshold))
        self.epoch += 1
        if training:
            self.saved_epoch = self.epoch
        return logits

    # ------------------------------------------------------------------ backward
    def _block_bwd(self, blk: BlockSpec, ga2, acts, x0, c0, x1, c1, gx_out0, gx_out1, cy0, N, S, lvl,
                   bn1_rows: int = 0, pool_dp=None):
        """Backward of one DoubleConv block. ga2: grad of block output (None: the second
        BN + ReLU backward was already done by its consumer, gY{lvl} holds dy2).  Writes the
        grad of the block input into gx_out0 (channels [0, cy0)) / gx_out1 (rest); None = skip.
        ``bn1_rows``: the second BatchNorm's backward partial rows are already in the stats
        buffer (written by pcms_maxpool_bwd_bn), only its finish + apply run here.  ``pool_dp``:
        they came from pcms_maxpool_bwd_bn_sums (ga2 holds the skip part only) and the apply
        adds the pooled gradient ``pool_dp`` itself (pcms_maxpool_bn_apply)."""
        b = self.bufs
        nvox = N * S[0] * S[1] * S[2]
        # the previous block's weight gradients (side stream) read this level's buffers until
        # joined (a decoder and an encoder block share gY / gZ / gA at one level)
        self._join_side()
        gY, gZ, gA = b[f"gY{lvl}"], b[f"gZ{lvl}"], b[f"gA{lvl}"]
        # BN1/ReLU backward -> dy2; its weight gradient on the side stream
        if ga2 is not None and bn1_rows:
            m = blk.b1.mod
            call("pcms_bn_relu_bwd_finish", self.code, ga2, acts["y2"], blk.b1.scale, blk.b1.shift, blk.b1.mean,
                 blk.b1.invstd, m.weight, b["stats"], bn1_rows, b["coef"], m.weight.grad, m.bias.grad,
                 gY if pool_dp is None else None, blk.b1.c, nvox, b["bnws"])
            if pool_dp is not None:
                call("pcms_maxpool_bn_apply", self.code, acts["y2"], blk.b1.scale, blk.b1.shift, blk.b1.mean,
                     blk.b1.invstd, b["coef"], pool_dp, ga2, gY, N, *S, blk.b1.c)
        elif ga2 is not None:
            self._bn_bwd(blk.b1, ga2, acts["y2"], gY, nvox)
        if ga2 is not None:
            self._grads_done(blk.b1.mod.weight, blk.b1.mod.bias)
        with self._side(lvl):
            if id(blk) in self._fwd_bnin:  # x = relu(bn0(y1)), applied in the kernel's staging (as the forward)
                call("pcms_conv3_wgrad_bnin", blk.c1.code, acts["y1"], blk.c0.cout, blk.b0.scale, blk.b0.shift, gY,
                     blk.c1.mod.weight.grad, b["dwt"], N, *S, blk.c1.cout, blk.c1.cin, self.wgrad_target,
                     int(self._gstore))
            else:
                call("pcms_conv3_wgrad", blk.c1.code, acts["a1"], blk.c0.cout, None, 0, gY, blk.c1.mod.weight.grad,
                     b["dwt"], N, *S, blk.c1.cout, blk.c1.cin, self.wgrad_target, int(self._gstore))
        self._grads_done(blk.c1.mod.weight, blk.c1.mod.bias)
        # dgrad conv1 -> grad of a1
        self._dgrad(blk.c1, gY, gA, None, blk.c1.cin, N, S)
        # BN0/ReLU backward -> dy1 (a second buffer: the side stream may still read gY)
        if blk is self.enc[0] and self.stem_sup & 2:
            # the stem: its BN0 apply runs inside the weight-gradient kernel (dy never stored)
            bn = blk.b0
            m = bn.mod
            call("pcms_bn_relu_bwd", self.code, gA, acts["y1"], bn.scale, bn.shift, bn.mean, bn.invstd, m.weight,
                 b["stats"], b["coef"], m.weight.grad, m.bias.grad, None, bn.c, nvox, b["bnws"])
            self._grads_done(m.weight, m.bias)
            with self._side(lvl), self._timed("stem_wgrad"):
                call("pcms_stem_wgrad_bn", x0, gA, acts["y1"], bn.scale, bn.shift, bn.mean, bn.invstd, b["coef"],
                     blk.c0.mod.weight.grad, b["dwt"], blk.c0.cin, N, *S)
            self._grads_done(blk.c0.mod.weight, blk.c0.mod.bias)
            return
        self._bn_bwd(blk.b0, gA, acts["y1"], gZ, nvox)
        self._grads_done(blk.b0.mod.weight, blk.b0.mod.bias)
        with self._side(lvl):
            if blk is self.enc[0] and self.stem_sup & 2:
                with self._timed("stem_wgrad"):
                    call("pcms_stem_wgrad", x0, gZ, blk.c0.mod.weight.grad, b["dwt"], blk.c0.cin, N, *S)
            else:
                call("pcms_conv3_wgrad", blk.c0.code, x0, c0, x1, c1, gZ, blk.c0.mod.weight.grad, b["dwt"], N,
                     *S, blk.c0.cout, blk.c0.cin, self.wgrad_target, int(self._gstore))
        self._grads_done(blk.c0.mod.weight, blk.c0.mod.bias)
        if gx_out0 is not None:
            self._dgrad(blk.c0, gZ, gx_out0, gx_out1, cy0, N, S)

    def _bn_bwd(self, bn: BNSpec, ga, y, gy, nvox):
        b = self.bufs
        m = bn.mod
        call("pcms_bn_relu_bwd", self.code, ga, y, bn.scale, bn.shift, bn.mean, bn.invstd, m.weight,
             b["stats"], b["coef"], m.weight.grad, m.bias.grad, gy, bn.c, nvox, b["bnws"])

    def _dgrad(self, cs: ConvSpec, gy, out0, out1, cy0, N, S):
        b = self.bufs
        nvox = N * S[0] * S[1] * S[2]
        splits = self._splits(N, S, cs.cout, cs.cin, cs.code)
        if splits == 1 and cs.dgrad16 is not None and query("pcms_conv3_big16_ok", N, *S, cs.cout, 0, cs.cin):
            call("pcms_conv3_fwd16", gy, cs.cout, None, 0, None, None, cs.dgrad16, None, out0, out1, cy0, None, 0,
                 N, *S, cs.cin)
        elif splits == 1:
            self._old_packs(cs)
            call("pcms_conv3_fwd", cs.code, gy, cs.cout, None, 0, cs.dgrad, None, out0, out1, cy0,
                 None, None, 0, N, *S, cs.cin, 1)
        elif cs.dgrad16 is not None and (sp16 := query("pcms_conv3_fwd16_split_ok", N, *S, cs.cout, 0, cs.cin)):
            acc = b["yacc"]
            if sp16 * nvox * cs.cin > acc.numel():
                raise RuntimeError("split-K workspace smaller than the 16x16x32 split form needs")
            call("pcms_conv3_fwd16_split", gy, cs.cout, None, 0, cs.dgrad16, acc, N, *S, cs.cin, sp16)
            call("pcms_split_epilogue", self.code, acc, sp16, None, out0, out1, cy0, None, cs.cin, nvox, 0)
        else:
            acc = b["yacc"]
            self._old_packs(cs)
            call("pcms_conv3_fwd", cs.code, gy, cs.cout, None, 0, cs.dgrad, None, out0, out1, cy0,
                 acc, None, 0, N, *S, cs.cin, splits)
            call("pcms_split_epilogue", self.code, acc, query("pcms_conv3_splits", cs.code, cs.cout, splits),
                 None, out0, out1, cy0, None, cs.cin, nvox, 0)

    def backward(self, dlogits: torch.Tensor):
        if self.saved_epoch != self.epoch:
            raise RuntimeError("UNet3D backward must follow its own training forward (the engine keeps "
                               "only the activations of the latest forward)")
        if self.buf_key[7:9] != (self.wgrad_target, self.split_target):
            raise RuntimeError("wgrad_target / split_target changed between the forward and its backward (the "
                               "workspaces were sized for the forward's values)")
        fresh = self.sync_params(full=False, fresh_ok=True)
        self._gstore = fresh
        if fresh:
            ranges, nr, mx = self._store_plan()
            call("pcms_fill_ranges", self.flat_g, ranges, nr, mx, 0.0)
        b = self.bufs
        S, C = b["S"], b["C"]
        N = self.buf_key[0]
        dlogits = dlogits.contiguous().float()
        oc = self.model.outc
        D, H, W = S[0]
        # head + the last decoder block's BN + ReLU backward in two passes over its y2 (the
        # forward's level-0 y2: under checkpointing the shared set still holds it, and the
        # recompute below rewrites the same bits); dy2 -> gY0
        bn = self.dec[3].b1
        m = bn.mod
        call("pcms_head_bn_bwd", self.code, self._dec_acts(0)["y2"], bn.scale, bn.shift, bn.mean, bn.invstd, m.weight,
             dlogits, oc.weight, oc.weight.grad, oc.bias.grad, b["redws"], b["stats"], b["coef"], m.weight.grad,
             m.bias.grad, b["gY0"], D * H * W, N, self.ncls, b["bnws"])
        self._grads_done(oc.weight, oc.bias)
        self._grads_done(m.weight, m.bias)  # the last decoder block's second BatchNorm (fused above)
        g = None
        # decoder, last block first
        for i in reversed(range(4)):
            l = 3 - i
            blk = self.dec[i]
            acts = self._dec_acts(l)
            self._join_side()  # the recompute rewrites the shared set the side stream may still read
            if self.buf_key[4]:
                self._block_fwd(blk, b[f"e{l}_x"], C[l], b[f"d{l}_u"], C[l], acts, N, S[l], True, recompute=True)
            gu = b[f"gU{l}"]
            self._block_bwd(blk, g, acts, b[f"e{l}_x"], C[l], b[f"d{l}_u"], C[l], b[f"gx{l}"], gu, C[l], N,
                            S[l], l)
            up = self.ups[i]
            _, dpack = self.convt_packs[i]
            hin = b["e4_x"] if i == 0 else b[f"d{l + 1}_a2"]
            # weight and bias gradients in one pass over gu (the bias sum over the ConvT output
            # box, F.pad's front offsets floor((S[l] - 2 S[l + 1]) / 2))
            with self._side(l, self.convt_wgrad_side):
                call("pcms_convt_wgrad_bias", self.code, hin, gu, up.weight.grad, up.bias.grad,
                     b["ctws_w"] if self.convt_wgrad_side else b["ctws"], b["redws"], N, *S[l + 1], up.in_channels,
                     up.out_channels, *S[l], 512)
            self._grads_done(up.weight, up.bias)
            gnext = b["gx4"] if i == 0 else b[f"gA{l + 1}"]
            call("pcms_convt_dgrad_ws", self.code, gu, dpack, gnext, b["ctws"], N, *S[l + 1], up.in_channels,
                 up.out_channels, *S[l])
            g = gnext
        # encoder, deepest first; gx{l} holds the skip gradient already (l < 4)
        rows, pool_dp = 0, None
        for l in reversed(range(5)):
            blk = self.enc[l]
            acts = {"y1": b[f"e{l}_y1"], "a1": b[f"e{l}_a1"], "y2": b[f"e{l}_y2"]}
            if l == 0:
                self._block_bwd(blk, b["gx0"], acts, b["xin"], self.cp, None, 0, None, None, 0, N, S[0], 0,
                                bn1_rows=rows, pool_dp=pool_dp)
            else:
                gp = b[f"gU{l}"]
                self._block_bwd(blk, b[f"gx{l}"], acts, b[f"pool{l}"], C[l - 1], None, 0, gp, None, C[l - 1], N,
                                S[l], l, bn1_rows=rows, pool_dp=pool_dp)
                # MaxPool3d backward + the next block's second BN-backward reduction, one pass
                # (fused form: the pooled gradient is added again by that block's BN apply, so
                # the block output's gradient gx{l-1} is not rewritten)
                bn = self.enc[l - 1].b1
                call("pcms_maxpool_bwd_bn_sums" if self.pool_bn_apply_fused else "pcms_maxpool_bwd_bn", self.code,
                     b[f"e{l - 1}_y2"], bn.scale, bn.shift, bn.mean, bn.invstd, gp, b[f"gx{l - 1}"], b["stats"], N,
                     *S[l - 1], C[l - 1])
                pool_dp = gp if self.pool_bn_apply_fused else None
                rows = query("pcms_maxpool_bwd_bn_rows", self.code, N, *S[l - 1], C[l - 1])
        self._join_side()  # every weight gradient before the optimizer / all-reduce wait
        self.saved_epoch = -1
