"""Train-step entry points mirroring ``src/train.py`` on the MI355X path.

* ``build_model`` -- the reference's config switch (train.py:329-470 / eval.py:66-198) building the
  HIP-backed ``FusionModel`` / ``VideoNet`` / ``WavLMAudioEncoder``.
* ``train_one_epoch`` -- same loop semantics as train.py:185-244 (zero_grad, forward, CE or late NLL,
  backward, Adam step), but losses/preds stay on the device (no per-step ``.item()`` host syncs).
* ``TrainStep`` -- one explicit step (the unit ``bench.py`` times), with the optional RCCL gradient
  all-reduce between backward and the optimizer.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import torch
from torch import nn

from .dist import GradAllReduce
from .fusion import FusionModel
from .losses import CrossEntropyLoss, LateNLLLoss, add_scaled
from .optim import FusedAdam
from .video import VideoNet
from .wavlm_audio import WavLMAudioEncoder


def build_model(num_classes: int, fusion: str, pretrained_video: bool = True, xattn_head: str = "concat",
                xattn_d_model: int = 128, xattn_heads: int = 4, xattn_attn_dropout: float = 0.1,
                xattn_stochastic_depth: float = 0.1, temporal_pooling: str = "mean", temporal_num_heads: int = 4,
                temporal_num_layers: int = 1, temporal_dropout: float = 0.1, audio_n_mels: int = 64,
                use_resnet_audio: bool = True, use_wavlm: bool = False, fusion_align_mode: str = "none",
                fusion_align_dim: int = 256, fusion_align_temperature: float = 0.07,
                xattn_use_emotion_prior: bool = False, xattn_emotion_prior_dim: int = 8,
                xattn_emotion_prior_hidden_dim: int = 64, xattn_emotion_prior_dropout: float = 0.1,
                forward_emotion_prior_flags: bool = False) -> nn.Module:
    """train.py:329-470.

    Reference quirk kept on purpose: the reference never forwards the ``xattn_use_emotion_prior*``
    flags to ``FusionModel`` (train.py:454-469, eval.py:182-197), so its checkpoints have no prior
    weights; pass ``forward_emotion_prior_flags=True`` to actually enable the prior-bias path.
    The mel ``AudioNet`` encoder (use_wavlm=False) is outside the north-star path.
    """
    if not use_wavlm and fusion in {"audio", "late", "concat", "gated", "xattn", "xattn_concat", "xattn_gated"}:
        raise NotImplementedError("mel AudioNet (use_wavlm=False) is out of scope; the MI355X path is WavLM")
    tp = dict(temporal_pooling=temporal_pooling, temporal_num_heads=temporal_num_heads,
              temporal_num_layers=temporal_num_layers, temporal_dropout=temporal_dropout)
    if fusion == "audio":
        return WavLMAudioEncoder(num_classes=num_classes, **tp)
    if fusion == "video":
        return VideoNet(num_classes=num_classes, pretrained=pretrained_video, **tp)
    audio = WavLMAudioEncoder(num_classes=num_classes, **tp)
    video = VideoNet(num_classes=num_classes, pretrained=pretrained_video, **tp)
    if fusion in {"late", "concat", "gated"}:
        return FusionModel(audio, video, num_classes=num_classes, mode=fusion, fusion_align_mode=fusion_align_mode,
                           fusion_align_dim=fusion_align_dim, fusion_align_temperature=fusion_align_temperature)
    if fusion in {"xattn", "xattn_concat", "xattn_gated"}:
        head = {"xattn_concat": "concat", "xattn_gated": "gated"}.get(fusion, xattn_head)
        prior = dict(xattn_use_emotion_prior=xattn_use_emotion_prior, xattn_emotion_prior_dim=xattn_emotion_prior_dim,
                     xattn_emotion_prior_hidden_dim=xattn_emotion_prior_hidden_dim,
                     xattn_emotion_prior_dropout=xattn_emotion_prior_dropout) if forward_emotion_prior_flags else {}
        return FusionModel(audio, video, num_classes=num_classes, mode="xattn", xattn_head=head, d_model=xattn_d_model,
                           num_heads=xattn_heads, audio_n_mels=768, xattn_attn_dropout=xattn_attn_dropout,
                           xattn_stochastic_depth=xattn_stochastic_depth, **tp, **prior)
    raise ValueError(f"Unknown fusion mode: {fusion}")


def _backward_order(model: nn.Module, params):
    """``params`` in the order their gradients become final in the backward (fusion head, the video encoder's
    head, ResNet18 layer4 .. stem, then the audio encoder), so the flat gradient buffer's prefix is what the
    early data-parallel bucket ships (dist.GradAllReduce).  Adam is per-parameter: the order changes nothing
    else."""
    names = {id(q): n for n, q in model.named_parameters()}

    def rank(q):
        n = names.get(id(q), "")
        if n.startswith("audio_model."):
            return (3, 0)
        if n.startswith("video_model.backbone."):
            parts = n.split(".")
            idx = int(parts[2])  # Sequential child: 0 conv1, 1 bn1, 4..7 layer1..4
            blk = (idx - 4) * 2 + int(parts[3]) if 4 <= idx <= 7 else -1
            return (2, -blk)
        if n.startswith("video_model."):
            return (1, 0)
        return (0, 0)

    return sorted(params, key=rank)  # stable: module order inside each rank


def build_optimizer(model: nn.Module, lr: float = 1e-3, weight_decay: float = 1e-4) -> FusedAdam:
    """train.py:899-902: Adam over every requires_grad parameter.  Parameters the configured mode never reaches
    (``FusionModel.unused_parameters``: audio_time_conv, the encoders' classifiers under xattn ...) get no
    gradient in the reference, so its Adam skips them on every step; they are left out of the flat buffers
    (and the data-parallel all-reduce) here, which is the same update."""
    params = build_optimizer_param_order(model)
    if not params:
        raise RuntimeError("No trainable parameters found for optimizer.")
    return FusedAdam(params, lr=lr, weight_decay=weight_decay)


def build_optimizer_param_order(model: nn.Module):
    """The used trainable parameters in flat-buffer (backward) order."""
    dead = {id(q) for q in getattr(model, "unused_parameters", lambda: [])()}
    return _backward_order(model, [p for p in model.parameters() if p.requires_grad and id(p) not in dead])



def _set_module_trainable(module: nn.Module, trainable: bool) -> None:
    for param in module.parameters():
        param.requires_grad = trainable


def set_video_backbone_trainable(video_model: nn.Module, unfreeze_blocks: int) -> None:
    """train.py:777-796: freeze the video branch, then unfreeze its last ``unfreeze_blocks`` parameterised
    backbone children (and its classifier)."""
    _set_module_trainable(video_model, False)
    if unfreeze_blocks <= 0:
        return
    backbone = getattr(video_model, "backbone", None)
    if not isinstance(backbone, nn.Sequential):
        _set_module_trainable(video_model, True)
        return
    parameterized = [m for m in backbone if len(list(m.parameters())) > 0]
    for m in parameterized[-unfreeze_blocks:]:
        _set_module_trainable(m, True)
    if hasattr(video_model, "classifier"):
        _set_module_trainable(video_model.classifier, True)


def apply_two_stage_freeze_policy(model: FusionModel, stage: int, unfreeze_wavlm_layers: int = 2,
                                  unfreeze_video_blocks: int = 1, unfreeze_audio: bool = True) -> None:
    """train.py:798-829 (defaults of --fusion_unfreeze_wavlm_layers / _video_blocks / _audio, train.py:629-648).
    Stage 1: fusion head only.  Stage 2: + the last WavLM layers (their backward runs on
    csrc/wavlm_train.hip) + the last video backbone blocks."""
    for name, param in model.named_parameters():
        if not name.startswith(("audio_model.", "video_model.")):
            param.requires_grad = True
    if stage == 1:
        _set_module_trainable(model.audio_model, False)
        _set_module_trainable(model.video_model, False)
        return
    if stage != 2:
        raise ValueError(f"Unsupported stage for two-stage training: {stage}")
    audio_model = model.audio_model
    if isinstance(audio_model, WavLMAudioEncoder):
        _set_module_trainable(audio_model, False)
        _set_module_trainable(audio_model.classifier, True)
        audio_model.unfreeze_backbone(max(0, int(unfreeze_wavlm_layers)))
    else:
        _set_module_trainable(audio_model, bool(unfreeze_audio))
    set_video_backbone_trainable(model.video_model, max(0, int(unfreeze_video_blocks)))


def build_fusion_stage_optimizer(model: nn.Module, stage: int, lr: float = 1e-3, audio_backbone_lr: float = 1e-5,
                                 video_backbone_lr: float = 1e-5, weight_decay: float = 1e-4) -> FusedAdam:
    """train.py:831-872: param groups fusion@lr, audio@audio_backbone_lr, video@video_backbone_lr."""
    fusion, audio, video = [], [], []
    dead = {id(q) for q in getattr(model, "unused_parameters", lambda: [])()}
    for name, param in model.named_parameters():
        if not param.requires_grad or id(param) in dead:
            continue
        (audio if name.startswith("audio_model.") else video if name.startswith("video_model.") else fusion).append(param)
    groups = []
    if stage == 1:
        if not fusion:
            raise RuntimeError("Stage-1 expects fusion parameters, but none are trainable.")
        groups.append({"params": fusion, "lr": lr})
    elif stage == 2:
        for ps, glr in ((fusion, lr), (audio, audio_backbone_lr), (video, video_backbone_lr)):
            if ps:
                groups.append({"params": _backward_order(model, ps), "lr": glr})
        if not groups:
            raise RuntimeError("Stage-2 expects trainable parameters, but none are trainable.")
    else:
        raise ValueError(f"Unsupported optimizer stage: {stage}")
    return FusedAdam(groups, lr=lr, weight_decay=weight_decay)

def make_loss(fusion_mode: str, label_smoothing: float = 0.0) -> nn.Module:
    """train.py:1030-1033."""
    return LateNLLLoss() if fusion_mode == "late" else CrossEntropyLoss(label_smoothing=label_smoothing)


# Early prefetch (FusionModel.queue_next_audio): the next batch's frozen audio encoder starts at the top of the
# step instead of before its backward (tests set EARLY_PREFETCH = False for the backward-only overlap).
EARLY_PREFETCH = True


class TrainStep:
    """One training step of train.py:200-228 on the HIP path: returns (loss, preds) as device tensors."""

    def __init__(self, model: nn.Module, optimizer: FusedAdam, loss_fn: nn.Module, fusion_mode: str,
                 grad_sync: Optional[GradAllReduce] = None, fusion_align_weight: float = 0.0):
        self.model, self.opt, self.loss_fn, self.mode = model, optimizer, loss_fn, fusion_mode
        self.grad_sync = grad_sync
        self.fusion_align_weight = float(fusion_align_weight)
        self.last_losses = None  # (cls_loss, contrastive_loss) device scalars of the last step

    def __call__(self, video: torch.Tensor, audio: torch.Tensor, labels: torch.Tensor,
                 next_audio: Optional[torch.Tensor] = None):
        """``next_audio``: the NEXT step's waveform batch, already on the device.  With a frozen audio
        encoder its forward is started on a side stream -- at the top of this step's xattn forward (early
        prefetch), else right after the forward -- so it overlaps this step's work
        (``FusionModel.prefetch_audio``); results are identical either way.  (A high-priority step stream was
        measured in round 2 and dropped: 5.50 vs 5.43 ms, profiles/r02c/ab_hiprio_*.json.)"""
        if not self.model.training:  # (a full module-tree walk; skipped when already in train mode)
            self.model.train()
        self.opt.zero_grad()
        early = EARLY_PREFETCH and next_audio is not None and hasattr(self.model, "queue_next_audio")
        if early:  # the forward starts it right after taking this batch's encoder output (overlaps the whole step)
            self.model.queue_next_audio(next_audio)
        if self.mode in {"audio", "video"}:
            outputs = self.model(audio if self.mode == "audio" else video)
        else:
            outputs = self.model(video, audio)
        cls_loss = loss = self.loss_fn(outputs, labels)
        align = None
        if self.mode != "late" and self.fusion_align_weight > 0.0 and hasattr(self.model, "pop_alignment_loss"):
            align = self.model.pop_alignment_loss()  # train.py:221-225
            if align is not None:
                loss = add_scaled(cls_loss, align, self.fusion_align_weight)
        self.last_losses = (cls_loss.detach(), align.detach() if align is not None else None)
        if early:
            next_audio = self.model.take_queued_audio()  # None when the forward issued it
        if next_audio is not None and hasattr(self.model, "prefetch_audio"):
            self.model.prefetch_audio(next_audio)
        loss.backward()
        if self.grad_sync is not None:
            self.grad_sync()
        self.opt.step()
        preds = getattr(self.loss_fn, "last_preds", None)  # the CE kernel's top-1 (train.py:216,220)
        if preds is None:
            raise RuntimeError("TrainStep needs a loss from losses.py (it writes the top-1 predictions)")
        return loss.detach(), preds


def train_one_epoch(model: nn.Module, loader, optimizer: FusedAdam, device: torch.device, loss_fn: nn.Module,
                    fusion_mode: str, fusion_align_weight: float = 0.0,
                    grad_sync: Optional[GradAllReduce] = None) -> Dict[str, float]:
    """train.py:185-244 (accuracy / macro-F1 computed once at the end, on the host).

    ``loader`` yields the reference's ``(video, audio, labels, meta)`` batches (ravdess.py:616, 654 through a
    DataLoader; ``data.ClipLoader`` yields the same); ``(video, audio, labels)`` is accepted too.  One batch of
    lookahead: the next batch's waveform starts its frozen-encoder forward during this step (TrainStep
    ``next_audio``), which changes no result."""
    step = TrainStep(model, optimizer, loss_fn, fusion_mode, grad_sync, fusion_align_weight=fusion_align_weight)
    losses, cls_losses, con_losses, preds, targets = [], [], [], [], []
    n = 0

    def unpack(batch):
        if not isinstance(batch, (tuple, list)) or len(batch) not in (3, 4):
            raise ValueError("loader batches must be (video, audio, labels[, meta])")
        return batch[0], batch[1].to(device), batch[2]

    it = iter(loader)
    nxt = next(it, None)
    nxt = unpack(nxt) if nxt is not None else None
    while nxt is not None:
        video, audio, labels = nxt
        video, labels = video.to(device), labels.to(device)
        nxt = next(it, None)  # one batch of lookahead: its audio feeds the encoder prefetch
        nxt = unpack(nxt) if nxt is not None else None
        nxt_audio = nxt[1] if nxt is not None else None
        loss, pred = step(video, audio, labels, next_audio=nxt_audio)
        losses.append(loss * labels.numel())
        cls_l, con_l = step.last_losses
        cls_losses.append(cls_l * labels.numel())
        if con_l is not None:
            con_losses.append(con_l * labels.numel())
        preds.append(pred)
        targets.append(labels)
        n += labels.numel()
    preds_t = torch.cat(preds).cpu()
    targets_t = torch.cat(targets).cpu()
    total = float(torch.stack(losses).sum().cpu()) / max(n, 1)
    cls_total = float(torch.stack(cls_losses).sum().cpu()) / max(n, 1)
    con_total = float(torch.stack(con_losses).sum().cpu()) / max(n, 1) if con_losses else 0.0
    acc = float((preds_t == targets_t).float().mean()) if n else 0.0
    return {"loss": total, "cls_loss": cls_total, "contrastive_loss": con_total, "acc": acc,
            "f1": macro_f1(preds_t, targets_t)}


def macro_f1(preds: torch.Tensor, targets: torch.Tensor) -> float:
    """sklearn f1_score(average='macro') over the labels present (utils/metrics.py:13-16)."""
    labels = torch.unique(torch.cat([preds, targets]))
    f1s = []
    for c in labels:
        tp = ((preds == c) & (targets == c)).sum().item()
        fp = ((preds == c) & (targets != c)).sum().item()
        fn = ((preds != c) & (targets == c)).sum().item()
        denom = 2 * tp + fp + fn
        f1s.append(0.0 if denom == 0 else 2 * tp / denom)
    return float(sum(f1s) / len(f1s)) if f1s else 0.0


def save_checkpoint(model: nn.Module, path, val_f1: float, config: Optional[dict] = None) -> None:
    """train.py:1141-1144 checkpoint format {"model", "val_f1", "config"} (state-dict keys identical to the
    reference's, so ``optimized_runtime.TorchModelRunner`` and the reference's loaders read it).  Tensors are
    moved to the host; after FusedAdam re-homing they are views of its flat buffers, so they are copied out."""
    state = {k: v.detach().to("cpu", copy=True) for k, v in model.state_dict().items()}
    torch.save({"model": state, "val_f1": float(val_f1), "config": dict(config or {})}, str(path))
