"""``VideoNet`` mirror (``src/models/video.py``) with the ResNet18 trunk on HIP kernels.

``backbone`` is an ``nn.Sequential`` with torchvision resnet18's children[:-1] at the same indices
(0 conv1, 1 bn1, 2 relu, 3 maxpool, 4..7 layer1..4, 8 avgpool), so state-dict keys
(``video_model.backbone.5.0.downsample.1.running_var`` ...) match reference checkpoints.  Its
forward is ONE autograd node running the explicit NHWC-bf16 schedule below (implicit-GEMM convs
with fused BatchNorm statistics, BN-apply(+residual)+ReLU passes, maxpool / avgpool), train-mode
BatchNorm with running-stat updates, and an explicit reverse schedule for backward.
Pretrained ImageNet weights are a network fetch in the reference (video.py:21); offline, the
trunk starts from random init (``pretrained`` is accepted and ignored with a warning).
"""
from __future__ import annotations

import os
import warnings
from typing import List

import torch
from torch import nn

from . import graphs as G
from . import kernels as K
from .nn_ops import hip_linear
from .optim import weight_version
from .temporal import TemporalPooler

S2D_CH = 16  # stem input: 2x2 space-to-depth of RGB (12 channels) padded to 16 (mer_pack_input_s2d)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, inplanes: int, planes: int, stride: int = 1, downsample: nn.Module = None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 3, stride, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = nn.Conv2d(planes, planes, 3, 1, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.downsample = downsample
        self.stride = stride


def _layer(inplanes, planes, stride):
    ds = None
    if stride != 1 or inplanes != planes:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes, 1, stride, bias=False), nn.BatchNorm2d(planes))
    return nn.Sequential(BasicBlock(inplanes, planes, stride, ds), BasicBlock(planes, planes))


def _init_resnet(module: nn.Module) -> None:
    """torchvision's resnet init: kaiming_normal_(fan_out, relu) convs, BN weight 1 / bias 0."""
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)


def _blocks(trunk) -> List[BasicBlock]:
    return [b for layer in (trunk[4], trunk[5], trunk[6], trunk[7]) for b in layer]


def _bn_tensors(bn: nn.BatchNorm2d):
    return bn.weight, bn.bias


class _TrunkFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, trunk, training, want_backward, *params):
        runner = trunk.graph_runner(x, training, want_backward)
        if runner is not None:
            feats, saved = runner.forward(x)
            # released by the backward, or when this graph is dropped without one (ModalityDropout cut)
            ctx.gen = runner.cur_gen
            ctx.token = runner.token(ctx.gen)
        else:
            feats, saved = trunk_forward(trunk, x, training)
        ctx.saved, ctx.trunk, ctx.training, ctx.runner = saved, trunk, training, runner
        return feats.view(feats.shape[0], feats.shape[1], 1, 1)

    @staticmethod
    def backward(ctx, dfeat):
        dfeat = dfeat.reshape(dfeat.shape[0], -1).contiguous().float()
        params = list(ctx.trunk.parameters())
        if ctx.runner is not None and ctx.runner.backward_graphable(params):
            grads = ctx.runner.backward(dfeat, params)
        else:
            grads = trunk_backward(ctx.trunk, ctx.saved, dfeat, ctx.training, hook=ctx.trunk.grad_ready_hook)
        if ctx.runner is not None:
            ctx.runner.release(ctx.gen)
        return (None, None, None, None, *[grads.get(id(q)) for q in params])


class _TrunkGraphs(G.PendingGuard):
    """Captured forward / backward hipGraphs of one (input shape, mode) of the trunk (graphs.py).

    Forward graph: (space-to-depth frames, packed just before the replay) -> ... -> avgpool, with the per-step
    weight packing and the BatchNorm
    running-stat updates inside it; its saved activations are graph-owned static tensors.  Backward:
    the whole reverse schedule, writing every parameter gradient straight into the optimizer's flat
    gradient buffer (``FusedAdam`` slots, fixed addresses); returned to autograd as fresh views.  With a
    gradient-ready hook registered (data parallelism) the backward is two graphs -- layer4, then layer3 ..
    stem -- and the hook runs between their replays, so the early all-reduce bucket overlaps the rest.
    """

    def __init__(self, trunk, training):
        super().__init__()
        self.trunk, self.training = trunk, training
        self.fwd = None
        self.bwd = None
        self.cur_gen = 0

    def forward(self, x):
        # the frames are packed to space-to-depth bf16 straight into the graph's static input (one launch before
        # the replay), not copied as fp32 into a static buffer and packed inside the graph
        if self.fwd is None:
            self.fwd = G.StaticGraph(lambda s: trunk_forward(self.trunk, x, self.training, force_pack=True, s2d=s),
                                     [s2d_input(x)])
        s2d = self.fwd.static_in[0]
        s2d_input(x, s2d)
        feats, saved = self.fwd.replay(s2d)
        return G.hand_out(feats), saved

    @staticmethod
    def backward_graphable(params) -> bool:
        return all(q.grad is None and getattr(q, "_mer_grad_slot", None) is not None
                   for q in params if q.requires_grad)

    def backward(self, dfeat, params):
        hook = self.trunk.grad_ready_hook
        split = SPLIT_BLOCK if hook is not None else 0
        if self.bwd is None or self.bwd[0] != split:
            _, saved = self.fwd.out
            tr, training = self.trunk, self.training
            tr.prepare_backward(dfeat.device)  # host-side setup (H2D copies) must not happen inside a capture
            if split:
                ga = G.StaticGraph(lambda d: trunk_backward_start(tr, saved, d, training, split, force_pack=True),
                                   [dfeat])
                gb = G.StaticGraph(lambda: trunk_backward_finish(tr, saved, ga.out, training, force_pack=True), [])
            else:
                ga = G.StaticGraph(lambda d: trunk_backward(tr, saved, d, training, force_pack=True), [dfeat])
                gb = None
            self.bwd = (split, ga, gb)
        _, ga, gb = self.bwd
        ga.replay(dfeat)
        if gb is not None:
            hook(self.trunk.split_params(split))
            gb.replay()
        from .fusion import grad_buffer  # fresh views of the flat-buffer slots the graph wrote
        return {id(q): grad_buffer(q) for q in params if q.requires_grad}


# First BasicBlock of the early gradient bucket: blocks 6, 7 = layer4 (8.4 M of the trunk's 11.2 M parameters)
SPLIT_BLOCK = 6


class ResNet18Trunk(nn.Sequential):
    """torchvision resnet18 children[:-1] (video.py:21-23) with a HIP forward."""

    def __init__(self):
        super().__init__(nn.Conv2d(3, 64, 7, 2, 3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
                         nn.MaxPool2d(3, 2, 1), _layer(64, 64, 1), _layer(64, 128, 2), _layer(128, 256, 2),
                         _layer(256, 512, 2), nn.AdaptiveAvgPool2d((1, 1)))
        _init_resnet(self)
        self._plans = {}
        self._force_pack = False
        self._graphs = G.GraphCache()
        self.grad_ready_hook = None  # fn(params): gradients of blocks >= SPLIT_BLOCK are final (dist.py)

    def prepare_backward(self, device) -> None:
        """Create the backward's lazily built device tables outside any graph capture: the transposed pack plan
        and the stem's space-to-depth weight-gradient index (a gradient-cut first step -- gated ModalityDropout
        -- can reach the first backward capture with neither built by an eager backward)."""
        self._pack_plan(True)
        self.stem_wgrad_table(device, WGRAD_DEFER)

    def stem_wgrad_table(self, device, deferred: bool) -> torch.Tensor:
        """The stem's space-to-depth weight-gradient table on ``device``: the slab-column -> 7x7-weight map of the
        deferred fold (``deferred``) or the gather index of the immediate one.  Built once (a pageable H2D copy
        that must not run inside a graph capture, hence prepare_backward)."""
        key = "_mer_stem_map" if deferred else "_mer_stem_idx"
        t = self.__dict__.get(key)
        if t is None or t.device != device:
            if G.capturing():
                raise RuntimeError("stem weight-gradient table built inside a graph capture; call prepare_backward")
            Kc, Cin, R, S = self[0].weight.shape
            t = self.__dict__[key] = (_stem_wgrad_map if deferred else _stem_wgrad_index)(R, S, Cin, device)
        return t

    def split_params(self, split: int):
        """Parameters whose gradients are final once the backward has passed BasicBlock ``split``."""
        return [q for b in _blocks(self)[split:] for q in b.parameters()]

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if not x.is_cuda:
            raise RuntimeError("ResNet18 trunk runs on the MI355X kernels; move the frames to the GPU")
        return _TrunkFn.apply(x.contiguous().float(), self, self.training, torch.is_grad_enabled(), *self.parameters())

    def graph_runner(self, x: torch.Tensor, training: bool, want_backward: bool = False):
        """The captured-graph runner for this input shape / mode, or None (eager) while warming up, during a
        capture, or for a second forward before the first one's backward (graphs.py)."""
        if G.capturing():
            return None
        key = (tuple(x.shape), bool(training), x.device.index, G.tensor_addresses(self), self.backward_stop())
        if not self._graphs.ready(key):
            return None
        r = self._graphs.get(key)
        if r is None:
            r = self._graphs.put(key, _TrunkGraphs(self, training))
        if r.pending:
            return None
        r.cur_gen = r.claim(bool(want_backward))
        return r

    def backward_stop(self) -> int:
        """Lowest BasicBlock index the backward must reach: -1 when the stem trains (full backward), else the
        first block with a trainable parameter (train.py:777-796 unfreezes only the last backbone children; the
        frames never need a gradient, so nothing below that block is computed), len(blocks) when frozen."""
        flags = tuple(q.requires_grad for q in self._param_list())
        cache = self.__dict__.get("_mer_bwd_stop")
        if cache is not None and cache[0] == flags:
            return cache[1]
        if any(q.requires_grad for m in (self[0], self[1]) for q in m.parameters()):
            stop = -1
        else:
            blocks = _blocks(self)
            stop = next((i for i, b in enumerate(blocks) if any(q.requires_grad for q in b.parameters())), len(blocks))
        self.__dict__["_mer_bwd_stop"] = (flags, stop)
        return stop

    def _param_list(self):
        lst = self.__dict__.get("_mer_params")
        if lst is None:
            lst = self.__dict__["_mer_params"] = list(self.parameters())
        return lst

    # ---- bf16 weight packing: all convs in one launch, re-done whenever a weight's value changes ----
    def _pack_plan(self, transpose: bool):
        """Persistent packed-weight buffers + the device descriptor table of one batched pack launch.
        Forward packs [K][R][S][Cp] for every conv (the stem in its space-to-depth 4x4 form); transposed packs
        [Cp][R][S][K] for every conv but the stem (the frames need no data gradient), as 64x64 tile transposes of
        the forward bf16 packs (mode 3: half the bytes of re-reading the fp32 weights; pack_all(True) refreshes
        the forward packs first if they are stale)."""
        convs = self.__dict__.get("_mer_convs")
        if convs is None:
            convs = self.__dict__["_mer_convs"] = [m for m in self.modules() if isinstance(m, nn.Conv2d)]
        fwd = None
        if transpose:
            convs = convs[1:]
            fwd = self._pack_plan(False)
        ptrs = tuple(c.weight.data_ptr() for c in convs) + ((id(fwd),) if fwd is not None else ())
        plan = self._plans.get(transpose)
        if plan is not None and plan["ptrs"] == ptrs:
            return plan
        dev = convs[0].weight.device
        outs, rows, first, blocks = {}, [], 0, 0
        for c in convs:
            Kc, C, R, S = c.weight.shape
            if C * R * S > 4608 or Kc > 512 or C > 512:  # the batched kernel's LDS tile / grid bounds
                raise ValueError(f"conv {tuple(c.weight.shape)} exceeds mer_pack_conv_weights' tile bounds")
            mode = int(transpose)
            if c is convs[0] and not transpose:  # the stem: space-to-depth 4x4 layout (mer_pack_input_s2d)
                mode, cp = 2, S2D_CH
                shape = (Kc, ((R + 2) // 2) * ((S + 2) // 2) * cp)
            else:
                cp = C
                shape = (cp, R * S * Kc) if transpose else (Kc, R * S * cp)
            buf = torch.empty(shape, device=dev, dtype=torch.bfloat16)
            outs[id(c)] = buf
            src = c.weight.data_ptr()
            if transpose and C % 64 == 0 and Kc % 64 == 0:
                mode, src = 3, fwd["outs"][id(c)].data_ptr()
            rows.append([src, buf.data_ptr(), Kc, C, R, S, cp, mode, blocks])
            first += buf.numel()
            # blocks: (tap, c tile, k tile) | (c, 64-k tile) | one per k
            blocks += (R * S * (C // 64) * (Kc // 64) if mode == 3 else cp * ((Kc + 63) // 64) if mode == 1
                       else Kc)
        plan = dict(convs=convs, ptrs=ptrs, outs=outs, total=first, blocks=blocks, vers=None, fwd=fwd,
                    desc=torch.tensor(rows, dtype=torch.int64).to(dev))
        self._plans[transpose] = plan
        return plan

    def pack_all(self, transpose: bool):
        """(Re-)pack every conv weight in one launch when any weight changed (always inside a capture)."""
        plan = self._pack_plan(transpose)
        vers = tuple(weight_version(c.weight) for c in plan["convs"])
        if plan["fwd"] is not None and plan["fwd"]["vers"] != tuple(weight_version(c.weight)
                                                                    for c in plan["fwd"]["convs"]):
            self.pack_all(False)  # the transposed packs read the forward packs
        if self._force_pack or vers != plan["vers"]:
            K.pack_conv_weights(plan["desc"], plan["blocks"])
            plan["vers"] = vers

    def packed(self, conv: nn.Conv2d, cp: int, transpose: bool):
        """The packed weight of ``conv`` (trunk_forward / trunk_backward refresh all packs on entry; a direct
        block-level call packs on first use)."""
        plan = self._pack_plan(transpose)
        if plan["vers"] is None:
            self.pack_all(transpose)
        buf = plan["outs"][id(conv)]
        if conv is plan["convs"][0] and not transpose:
            return buf  # the space-to-depth stem pack [K][4][4][16]
        if (buf.shape[0] if transpose else buf.shape[1] // (conv.weight.shape[2] * conv.weight.shape[3])) != cp:
            raise ValueError(f"packed weight channel padding {cp} does not match the plan")
        return buf


def _bn_forward(bn: nn.BatchNorm2d, c: torch.Tensor, stats, training: bool, rows=None):
    """``rows``: the statistics rows the conv wrote (K.conv_fwd's return: one per workgroup on the halo kernel)."""
    C = c.shape[-1]
    ms = torch.empty(C, 2, device=c.device, dtype=torch.float32)
    M = c.numel() // C
    if training:
        mom = 0.1 if bn.momentum is None else bn.momentum
        K.bn_finalize(stats, M, bn.eps, mom, ms, bn.running_mean, bn.running_var, bn.num_batches_tracked, rows=rows)
    else:
        K.bn_finalize(None, M, bn.eps, 0.0, ms, bn.running_mean, bn.running_var)
    return ms


def _fwd_stat_floats(trunk, N: int, H: int, W: int) -> int:
    """Floats of every conv's forward BatchNorm statistics (MER_BN_STAT_ROWS(M) x C x 2) for [N,3,H,W] frames."""
    h, w = H // 2, W // 2  # stem conv output (space-to-depth form)
    total = K.bn_stat_rows(N * h * w) * trunk[0].out_channels * 2
    h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1  # maxpool
    for blk in _blocks(trunk):
        s = blk.stride
        h, w = (h + 2 - 3) // s + 1, (w + 2 - 3) // s + 1
        convs = [blk.conv1, blk.conv2] + ([blk.downsample[0]] if blk.downsample is not None else [])
        total += sum(K.bn_stat_rows(N * h * w) * c.out_channels * 2 for c in convs)
    return total


class _StatsArena:
    """One zeroed buffer for all BatchNorm partial sums of a trunk pass: one memset instead of one per BN.
    Forward: per-row-tile statistics rows (``take(C, M=...)``, float[MER_BN_STAT_ROWS(M)][C][2], sized by
    ``_fwd_stat_floats``); backward: striped reduction rows (float[MER_BN_STAT_PARTS][C][2] or [C][2])."""

    def __init__(self, trunk, device, factor: int = 1, floats: int = 0, zero: bool = True):
        total = sum(m.out_channels for m in trunk.modules() if isinstance(m, nn.Conv2d))
        n = floats if floats else factor * K.BN_STAT_PARTS * 2 * total
        # zero=False: every row a reader folds is written first (the forward statistics of default-variant convs, whose
        # exact row counts K.conv_fwd returns) -- no 22.6 MB memset on the trunk stream at B = 32
        self.buf = (torch.zeros if zero else torch.empty)(n, device=device, dtype=torch.float32)
        self.off = 0

    def take(self, C, parts=None, M=None):
        if M is not None:
            parts = K.bn_stat_rows(M)
        parts = K.BN_STAT_PARTS if parts is None else parts
        n = parts * 2 * C
        if self.off + n > self.buf.numel():
            raise RuntimeError("BatchNorm statistics arena exhausted")
        t = self.buf[self.off:self.off + n].view(parts, C, 2) if parts > 1 else self.buf[self.off:self.off + n].view(C, 2)
        self.off += n
        return t


def _check_stem(conv1, C, H, W):
    if tuple(conv1.weight.shape[1:]) != (C, 7, 7) or conv1.stride != (2, 2) or conv1.padding != (3, 3) \
            or C > 4 or H % 2 or W % 2:
        raise ValueError("the space-to-depth stem expects conv1 = 7x7/s2/p3 on <= 4 channels and even H, W")


def _stem_wgrad_index(R: int, S: int, C: int, device) -> torch.Tensor:
    """Flat index into a [16][Ro][So] space-to-depth weight gradient for every (c, r, s) of the 7x7 one."""
    So = (S + 2) // 2
    Ro = (R + 2) // 2
    idx = torch.empty(C, R, S, dtype=torch.int64)
    for c in range(C):
        for r in range(R):
            for s_ in range(S):
                ry, dy = divmod(r + 1, 2)
                rx, dx = divmod(s_ + 1, 2)
                idx[c, r, s_] = ((dy * 2 + dx) * C + c) * Ro * So + ry * So + rx
    return idx.view(-1).to(device)


def _stem_wgrad_map(R: int, S: int, C: int, device) -> torch.Tensor:
    """int32 [Ro*So*16]: for each column (tap, s2d channel) of the stem's wgrad slabs, the flat (c, r, s) index of
    the 7x7 weight it is, or -1 (the zero-padded taps / channels); the inverse of _stem_wgrad_index."""
    So, Ro = (S + 2) // 2, (R + 2) // 2
    m = torch.full((Ro * So * S2D_CH,), -1, dtype=torch.int32)
    for c in range(C):
        for r in range(R):
            for s_ in range(S):
                ry, dy = divmod(r + 1, 2)
                rx, dx = divmod(s_ + 1, 2)
                m[(ry * So + rx) * S2D_CH + (dy * 2 + dx) * C + c] = (c * R + r) * S + s_
    return m.to(device)


def _conv_bn(trunk, conv, bn, x, stride, pad, training, arena=None, rs=None, defer=False):
    """conv (+ fused batch stats) -> (conv output, (mean, rstd)); ``defer`` (train mode): (output, stats, rows)."""
    Kc, _, R, S = conv.weight.shape
    if rs is not None:
        R, S = rs
    N, H, W, C = x.shape
    Ho, Wo = (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1
    y = torch.empty(N, Ho, Wo, Kc, device=x.device, dtype=torch.bfloat16)
    stats = None
    if training:
        M = N * Ho * Wo
        stats = arena.take(Kc, M=M) if arena is not None else K.bn_stats_buffer(Kc, x.device, M)
    rows = K.conv_fwd(x, trunk.packed(conv, C, False), y, stats, R, S, stride, pad)
    if defer:  # the caller finalizes (a paired launch): (output, its statistics, rows written)
        return y, stats, rows
    return y, _bn_forward(bn, y, stats, training, rows)


def _bn_forward_pair(bns, ys, stats, rows):
    """Two train-mode BatchNorm finalizes in one launch (K.bn_finalize_pair) -> their (mean, rstd) tables."""
    recs, out = [], []
    for bn, y, st, r in zip(bns, ys, stats, rows):
        C = y.shape[-1]
        ms = torch.empty(C, 2, device=y.device, dtype=torch.float32)
        if (0.1 if bn.momentum is None else bn.momentum) != (0.1 if bns[0].momentum is None else bns[0].momentum) \
                or bn.eps != bns[0].eps:
            raise ValueError("paired BatchNorm finalize needs one eps / momentum")
        recs.append((st, y.numel() // C, ms, bn.running_mean, bn.running_var, bn.num_batches_tracked, r))
        out.append(ms)
    K.bn_finalize_pair(recs[0], recs[1], bns[0].eps, 0.1 if bns[0].momentum is None else bns[0].momentum)
    return out


@torch.no_grad()
def block_forward(trunk, blk: BasicBlock, x: torch.Tensor, training: bool, arena=None):
    """BasicBlock (torchvision): relu(bn2(conv2(relu(bn1(conv1(x))))) + [bn_d(conv_d(x)) | x])."""
    s = blk.stride
    bc1, bms1 = _conv_bn(trunk, blk.conv1, blk.bn1, x, s, 1, training, arena)
    ba1 = torch.empty_like(bc1)
    K.bn_apply(bc1, bms1, blk.bn1.weight, blk.bn1.bias, ba1, relu=True)
    dbn = blk.downsample[1] if blk.downsample is not None else None
    paired = dbn is not None and training and BN_FIN_PAIR
    if paired:  # conv2 and the downsample conv first, then both BatchNorms' finalizes in one launch
        bc2, st2, r2 = _conv_bn(trunk, blk.conv2, blk.bn2, ba1, 1, 1, training, arena, defer=True)
        cd, std, rd = _conv_bn(trunk, blk.downsample[0], dbn, x, s, 0, training, arena, defer=True)
        bms2, msd = _bn_forward_pair((blk.bn2, dbn), (bc2, cd), (st2, std), (r2, rd))
    else:
        bc2, bms2 = _conv_bn(trunk, blk.conv2, blk.bn2, ba1, 1, 1, training, arena)
    out = torch.empty_like(bc2)
    if blk.downsample is not None:
        if not paired:
            cd, msd = _conv_bn(trunk, blk.downsample[0], blk.downsample[1], x, s, 0, training, arena)
        K.bn_apply(bc2, bms2, blk.bn2.weight, blk.bn2.bias, out, relu=True, res=cd, ms2=msd, gamma2=dbn.weight,
                   beta2=dbn.bias)
    else:
        cd = msd = None
        K.bn_apply(bc2, bms2, blk.bn2.weight, blk.bn2.bias, out, relu=True, res=x)
    return out, (x, bc1, bms1, ba1, bc2, bms2, cd, msd, out)


class _ForcePack:
    """Inside a graph capture every weight pack must be a captured kernel (the graph replays it each step),
    so the version-keyed pack cache is bypassed."""

    def __init__(self, trunk, on):
        self.trunk, self.on = trunk, on

    def __enter__(self):
        self.prev = self.trunk._force_pack
        self.trunk._force_pack = self.on or self.prev

    def __exit__(self, *exc):
        self.trunk._force_pack = self.prev


@torch.no_grad()
def trunk_forward(trunk: ResNet18Trunk, video: torch.Tensor, training: bool, force_pack: bool = False,
                  s2d: torch.Tensor = None):
    """``s2d``: the frames already packed by ``s2d_input`` (``video`` then only gives the shape) -- the captured
    forward graph takes the packed frames as its static input, so the per-step fp32 frame copy is not needed."""
    with _ForcePack(trunk, force_pack):
        return _trunk_forward(trunk, video, training, s2d)


def s2d_input(video: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """fp32 NCHW frames -> the stem's bf16 space-to-depth input [N][H/2+3][W/2+3][S2D_CH] (mer_pack_input_s2d)."""
    N, C, H, W = video.shape
    video = video.float().contiguous()
    if out is None:
        out = torch.empty(N, H // 2 + 3, W // 2 + 3, S2D_CH, device=video.device, dtype=torch.bfloat16)
    K.pack_input_s2d(video, out)
    return out


def _trunk_forward(trunk: ResNet18Trunk, video: torch.Tensor, training: bool, s2d: torch.Tensor = None):
    trunk.pack_all(transpose=False)
    N, C, H, W = video.shape
    dev = video.device
    bf = torch.bfloat16
    conv1, bn1 = trunk[0], trunk[1]
    _check_stem(conv1, C, H, W)
    # stem conv 7x7/s2/p3 as a 4x4/s1/p0 conv on the 2x2 space-to-depth frames (K = 256, not 7*7*8)
    if s2d is None:
        x0 = s2d_input(video)
    else:
        if tuple(s2d.shape) != (N, H // 2 + 3, W // 2 + 3, S2D_CH) or s2d.dtype != bf:
            raise ValueError(f"packed frames {tuple(s2d.shape)} do not match video {tuple(video.shape)}")
        x0 = s2d
    # (not zeroed when the finalizes read only written rows: same-box +0.1 %, profiles/r06/step_ab_fwd_rows_exact)
    arena = _StatsArena(trunk, dev, floats=_fwd_stat_floats(trunk, N, H, W), zero=not K.PARTIAL_ROWS) \
        if training else None
    c1, ms1 = _conv_bn(trunk, conv1, bn1, x0, 1, 0, training, arena, rs=(4, 4))
    Hp, Wp = (c1.shape[1] - 1) // 2 + 1, (c1.shape[2] - 1) // 2 + 1
    p1 = torch.empty(N, Hp, Wp, c1.shape[-1], device=dev, dtype=bf)
    arg = torch.empty(N, Hp, Wp, c1.shape[-1], device=dev, dtype=torch.uint8)
    K.stem_bnrelu_maxpool(c1, ms1, bn1.weight, bn1.bias, p1, arg)  # bn1 + relu + maxpool, activation not stored
    saved = {"stem": (x0, c1, ms1, arg), "blocks": []}
    x = p1
    for blk in _blocks(trunk):
        x, sv = block_forward(trunk, blk, x, training, arena)
        saved["blocks"].append(sv)
    feats = torch.empty(N, x.shape[-1], device=dev, dtype=torch.float32)
    K.avgpool_fwd(x, feats)
    saved["final"] = x
    return feats, saved


def _grad(param, grads):
    from .fusion import grad_buffer

    if not param.requires_grad:
        return None
    g = grads.get(id(param))
    if g is None:
        g = grad_buffer(param)
        grads[id(param)] = g
    return g


def _bn_bwd(g, mask, x, ms, bn, red, grads, training):
    """BatchNorm backward apply given the collapsed reduction red[C,2] = (sum g, sum g*xhat)."""
    dx = torch.empty_like(x)
    K.bn_bwd_apply(g, mask, x, ms, bn.weight, red, dx, _grad(bn.weight, grads), _grad(bn.bias, grads), training)
    return dx


def _block_bwd_floats(sv) -> int:
    """Arena floats for one block_backward: its bn1 reduction rows, two bn_bwd_reduce workspaces and the
    fused reductions of an upstream block's bn2 / downsample BN at the block input's resolution."""
    xin, bc1, _, ba1, bc2, _, _, _, out = sv
    C1, C2, Cin = bc1.shape[-1], bc2.shape[-1], xin.shape[-1]
    return 2 * (K.bn_red_rows(ba1.numel() // C1) * C1 + 2 * K.BN_RED_WS_ROWS * C2 + C2 * 2
                + 2 * K.bn_red_rows(xin.numel() // Cin) * Cin)


def _bnr_target(blk_sv, blk, arena):
    """The fused-reduction target for a gradient flowing into ``blk``'s output: its bn2 (and downsample
    BN) read g = grad * (out > 0); returns (bnr tuple for conv_dgrad, partial buffers)."""
    xin, bc1, bms1, ba1, bc2, bms2, cd, msd, out = blk_sv
    C2 = bc2.shape[-1]
    rows = K.bn_red_rows(out.numel() // C2)  # one row per dgrad output row tile (+ scratch)
    red2 = arena.take(C2, parts=rows)
    if cd is None:
        return (out, bc2, bms2, red2), (red2, None)
    redd = arena.take(C2, parts=rows)
    return (out, bc2, bms2, red2, cd, msd, redd), (red2, redd)


# Deferred weight-gradient folds (tests set WGRAD_DEFER = False to fold after every wgrad): the wgrad launches leave
# their split-K slabs and the segment's join folds them all in one mer_wgrad_fold_batch launch -- ~30 launches of
# 5-12 us each off the critical stream per step (the stem's zero / gather / add included).  (Round 3 also measured
# the weight gradients on a third stream and folding after every N blocks: both slower or inside the noise, removed.)
WGRAD_DEFER = True
# A stride-2 block's bn2 and downsample-BN backward applies in one pass over the shared gradient and mask
# (mer_bn_bwd_apply2, bit-identical; 3 x 4 fewer bytes per element and one launch less per stride-2 block; the
# same-box step did not move measurably: 211.51 vs 211.74 steps/s, profiles/r06/step_ab_fold_b8)
BN_BWD_PAIR = True
# A stride-2 block's bn2 and downsample-BN statistics folds paired into one launch, forward (mer_bn_finalize_rows2)
# and backward (mer_partials_sum2)
BN_FIN_PAIR = True  # same-box step +0.59 % (profiles/r06/step_ab_fin_pair)
# The deferred weight-gradient folds flushed at the end of every ResNet layer (every second BasicBlock) instead of once
# after all blocks: each fold reads slabs written a layer earlier (more of them still in the 256 MB MALL), three
# launches more per step; same-box +0.27 % (profiles/r06/step_ab_fold_per_layer)
FOLD_EVERY = 2
# The downsample's input gradient fused into conv1's stride-2 dgrad (mer_conv_dgrad_ds): +1.2 % same-box vs the
# separate 1x1 dgrad whose bf16 output the 3x3 dgrad read back as its residual (profiles/r04/ab_runs.txt)
FUSED_DS_DGRAD = True


class _WgradLane:
    """The weight-gradient launches of one backward (graph) segment and their deferred folds, flushed at join()."""

    def __init__(self, device):
        self.folds = K.WgradFolds() if WGRAD_DEFER else None

    def run(self, fn, *reads, block=None):
        fn()

    def join(self):
        if self.folds is not None:
            self.folds.flush()


@torch.no_grad()
def block_backward(trunk, blk: BasicBlock, sv, dx: torch.Tensor, grads, training: bool = True, pre=None,
                   prev=None, arena=None, lane=None, bidx=None):
    """Reverse of block_forward given dx = dL/d(block output); returns dL/d(block input).

    ``pre``: this block's bn2 / downsample-BN reductions already accumulated by the producer of ``dx``
    (partial buffers from the next block's fused dgrad), else they are reduced here.  ``prev``: the
    (saved, block) of the preceding block, whose reductions this block's input-gradient dgrad fuses.
    """
    dev = dx.device
    xin, bc1, bms1, ba1, bc2, bms2, cd, msd, out = sv
    if arena is None:  # standalone call: room for this block's own reductions and one upstream target
        arena = _StatsArena(trunk, dev, floats=_block_bwd_floats(sv))
    own_lane = lane is None
    if own_lane:
        lane = _WgradLane(dev)
    g_out = dx
    s = blk.stride
    C2 = bc2.shape[-1]
    if pre is not None:  # (red2 rows, downsample-BN rows, rows the producing dgrad wrote)
        if cd is not None and BN_FIN_PAIR:
            red2, redd = K.partials_sum_pair(pre[0], torch.empty(C2, 2, device=dev, dtype=torch.float32), pre[1],
                                             torch.empty(C2, 2, device=dev, dtype=torch.float32), pre[2])
        else:
            red2 = K.partials_sum(pre[0], torch.empty(C2, 2, device=dev, dtype=torch.float32), pre[2])
            redd = K.partials_sum(pre[1], torch.empty(C2, 2, device=dev, dtype=torch.float32), pre[2]) \
                if cd is not None else None
    else:
        red2 = arena.take(C2, parts=1)
        K.bn_bwd_reduce(g_out, out, bc2, bms2, red2, arena.take(C2, parts=K.BN_RED_WS_ROWS))
        redd = None
        if cd is not None:
            redd = arena.take(C2, parts=1)
            K.bn_bwd_reduce(g_out, out, cd, msd, redd, arena.take(C2, parts=K.BN_RED_WS_ROWS))
    if cd is not None and BN_BWD_PAIR:  # bn2 and the downsample BN read the same gradient and mask: one pass
        dc2, dcd = torch.empty_like(bc2), torch.empty_like(cd)
        bd = blk.downsample[1]
        K.bn_bwd_apply2(g_out, out, bc2, bms2, blk.bn2.weight, red2, dc2, _grad(blk.bn2.weight, grads),
                        _grad(blk.bn2.bias, grads), cd, msd, bd.weight, redd, dcd, _grad(bd.weight, grads),
                        _grad(bd.bias, grads), training)
    else:
        dc2 = _bn_bwd(g_out, out, bc2, bms2, blk.bn2, red2, grads, training)
        dcd = _bn_bwd(g_out, out, cd, msd, blk.downsample[1], redd, grads, training) if cd is not None else None
    # conv2 (its dgrad also reduces bn1's backward sums: g = da1 * (ba1 > 0))
    w2 = _grad(blk.conv2.weight, grads)
    if w2 is not None:
        lane.run(lambda: K.conv_wgrad(ba1, dc2, w2, 3, 3, 1, 1, defer=lane.folds), ba1, dc2, w2, block=bidx)
    da1 = torch.empty_like(ba1)
    C1 = bc1.shape[-1]
    red1p = arena.take(C1, parts=K.bn_red_rows(ba1.numel() // C1))
    rows1 = K.conv_dgrad(dc2, trunk.packed(blk.conv2, C2, True), da1, 3, 3, 1, 1, bnr=(ba1, bc1, bms1, red1p))
    red1 = K.partials_sum(red1p, torch.empty(C1, 2, device=dev, dtype=torch.float32), rows1)
    dc1 = _bn_bwd(da1, ba1, bc1, bms1, blk.bn1, red1, grads, training)
    # conv1 (+ downsample) -> dx of the block input (+ the preceding block's bn2 / downsample reductions)
    w1 = _grad(blk.conv1.weight, grads)
    if w1 is not None:
        lane.run(lambda: K.conv_wgrad(xin, dc1, w1, 3, 3, s, 1, defer=lane.folds), xin, dc1, w1, block=bidx)
    dxin = torch.empty_like(xin)
    Cin = xin.shape[-1]
    bnr, nxt = _bnr_target(prev[0], prev[1], arena) if prev is not None else (None, None)
    if cd is not None:
        wd = _grad(blk.downsample[0].weight, grads)
        if wd is not None:
            lane.run(lambda: K.conv_wgrad(xin, dcd, wd, 1, 1, s, 0, defer=lane.folds), xin, dcd, wd, block=bidx)
        if FUSED_DS_DGRAD and s == 2:  # the downsample's input gradient as an extra K segment of conv1's dgrad
            rows = K.conv_dgrad(dc1, trunk.packed(blk.conv1, Cin, True), dxin, 3, 3, s, 1, bnr=bnr,
                                ds=(dcd, trunk.packed(blk.downsample[0], Cin, True)))
        else:
            dxd = torch.empty_like(xin)
            K.conv_dgrad(dcd, trunk.packed(blk.downsample[0], Cin, True), dxd, 1, 1, s, 0)
            rows = K.conv_dgrad(dc1, trunk.packed(blk.conv1, Cin, True), dxin, 3, 3, s, 1, residual=dxd, bnr=bnr)
    else:
        rows = K.conv_dgrad(dc1, trunk.packed(blk.conv1, Cin, True), dxin, 3, 3, s, 1, residual=g_out, mask=out,
                            bnr=bnr)
    if own_lane:
        lane.join()
    return dxin, (nxt + (rows,) if nxt is not None else None)


@torch.no_grad()
def trunk_backward(trunk: ResNet18Trunk, saved, dfeat: torch.Tensor, training: bool = True, force_pack: bool = False,
                   hook=None):
    """Whole reverse schedule -> {id(param): grad}.  ``hook(params)`` (data parallelism) is called once the
    gradients of blocks >= SPLIT_BLOCK are enqueued, before the rest of the backward."""
    split = SPLIT_BLOCK if hook is not None else 0
    state = trunk_backward_start(trunk, saved, dfeat, training, split, force_pack=force_pack)
    if hook is not None:
        hook(trunk.split_params(split))
    return trunk_backward_finish(trunk, saved, state, training, force_pack=force_pack)


@torch.no_grad()
def trunk_backward_start(trunk, saved, dfeat, training, split, force_pack=False):
    """avgpool backward and BasicBlocks [max(split, stop), 8) in reverse; returns the state the rest needs."""
    with _ForcePack(trunk, force_pack):
        trunk.pack_all(transpose=True)
        dev = dfeat.device
        x = saved["final"]
        dx = torch.empty_like(x)
        K.avgpool_bwd(dfeat, dx)
        svs = saved["blocks"]
        # every backward BatchNorm reduction buffer of this pass: one memset
        # (still zeroed: leaving it unzeroed -- every row a fold reads is written first, the dgrads' reduction row
        # counts being exact -- measured +0.06 %, inside the noise, profiles/r06/step_ab_bwd_rows_exact)
        arena = _StatsArena(trunk, dev, floats=sum(_block_bwd_floats(sv) for sv in svs) + 2 * K.BN_RED_WS_ROWS * 64 * 2)
        state = dict(dx=dx, pre=None, grads={}, arena=arena, i=len(svs) - 1, lane=_WgradLane(dev))
        _backward_blocks(trunk, saved, state, max(split, trunk.backward_stop(), 0), training)
        state["lane"].join()  # the early-bucket hook (or the next graph segment) sees final layer4 gradients
        return state


def _backward_blocks(trunk, saved, state, lo, training):
    blocks, svs = _blocks(trunk), saved["blocks"]
    while state["i"] >= lo:
        i = state["i"]
        prev = (svs[i - 1], blocks[i - 1]) if i > 0 else None
        state["dx"], state["pre"] = block_backward(trunk, blocks[i], svs[i], state["dx"], state["grads"], training,
                                                   pre=state["pre"], prev=prev, arena=state["arena"],
                                                   lane=state["lane"], bidx=i)
        if FOLD_EVERY and i % FOLD_EVERY == 0 and i > 0:
            state["lane"].join()
        state["i"] = i - 1


@torch.no_grad()
def trunk_backward_finish(trunk, saved, state, training, force_pack=False):
    """The remaining BasicBlocks and the stem; returns {id(param): grad}."""
    with _ForcePack(trunk, force_pack):
        stop = trunk.backward_stop()
        _backward_blocks(trunk, saved, state, max(stop, 0), training)
        grads, arena, dx = state["grads"], state["arena"], state["dx"]
        if stop >= 0:  # stem and the blocks below `stop` frozen (stage-2 video tail): nothing more is needed
            state["lane"].join()
            return grads
        dev = dx.device
        # stem: maxpool -> bn1/relu -> conv1 (no data gradient for the frames)
        x0, c1, ms1, arg = saved["stem"]
        bn1 = trunk[1]
        red = arena.take(c1.shape[-1], parts=1)
        dc1 = torch.empty_like(c1)  # maxpool + relu + bn1 backward in one reduction pass and one apply pass
        K.stem_pool_bn_bwd(dx, arg, c1, ms1, bn1.weight, bn1.bias, red, dc1, _grad(bn1.weight, grads),
                           _grad(bn1.bias, grads), training, workspace=arena.take(c1.shape[-1], parts=K.BN_RED_WS_ROWS))
        w = _grad(trunk[0].weight, grads)
        if w is not None:  # wgrad of the 4x4 space-to-depth form, then gathered back to [64][3][7][7]
            Kc, Cin, R, S = trunk[0].weight.shape
            Ro, So = (R + 2) // 2, (S + 2) // 2
            folds = state["lane"].folds
            if folds is not None:  # slab column (tap, s2d channel) folds straight into the 7x7 weight
                K.conv_wgrad(x0, dc1, w, Ro, So, 1, 0, defer=folds, dw_map=trunk.stem_wgrad_table(dev, True))
            else:
                ws2d = torch.empty(Kc, S2D_CH, Ro, So, device=dev, dtype=torch.float32)
                ws2d.zero_()
                K.conv_wgrad(x0, dc1, ws2d, Ro, So, 1, 0)
                idx = trunk.stem_wgrad_table(dev, False)
                w.add_(ws2d.view(Kc, -1).index_select(1, idx).view_as(w))
        state["lane"].join()
        return grads


class VideoNet(nn.Module):
    """video.py:10-44 -- same constructor and encode/forward API."""

    def __init__(self, num_classes: int, pretrained: bool = True, temporal_pooling: str = "mean",
                 temporal_num_heads: int = 4, temporal_num_layers: int = 1, temporal_dropout: float = 0.1) -> None:
        super().__init__()
        if pretrained:
            warnings.warn("ImageNet weights are a network fetch in the reference (video.py:21); building the "
                          "resnet18 trunk from random init offline")
        self.backbone = ResNet18Trunk()
        self.embedding_dim = 512
        self.temporal_pool = TemporalPooler(self.embedding_dim, temporal_pooling, temporal_num_heads,
                                            temporal_num_layers, temporal_dropout)
        self.classifier = nn.Linear(self.embedding_dim, num_classes)

    def encode(self, x: torch.Tensor) -> torch.Tensor:
        b, t, c, h, w = x.shape
        feat = self.backbone(x.view(b * t, c, h, w)).view(b, t, self.embedding_dim)
        return self.temporal_pool(feat)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return hip_linear(self.encode(x), self.classifier)
