"""Convolutions on the CDNA4 kernels.

* ResNet stem (3 -> 64, 7x7, stride 2, pad 3): csrc/conv_stem.hip, bf16 channels-last forward
  and weight gradient with the image rows staged once per output row in LDS (channel dim padded
  3 -> 4 so every im2col operand is one aligned 16-byte LDS read).
* Every other convolution with C, K multiples of 64 (all of ResNet-50's bottleneck convs):
  csrc/conv_igemm.hip implicit GEMM -- the forward (with the following BatchNorm's batch
  statistics emitted from the epilogue, so BN skips its statistics pass) and the stride-1 input
  gradient (forward conv of dY with the flipped, transposed weights), and the weight gradient
  (pixel-split MFMA kernel with transposed LDS reads + deterministic split reduction).  The
  strided input gradient stays on MIOpen.  Tile configurations are picked per layer shape by
  timing every candidate once (MIOpen / hipBLASLt included for the gradients), like MIOpen's own
  find step.

Anything else -- other shapes, fp32 inputs, modules with hooks or parametrizations -- runs the
module's own convolution (MIOpen).
"""

import contextlib
import time
import os
from typing import Callable, Dict, Iterator, List, Optional, Tuple

import torch
from torch import nn


class _StemConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, want_stats):
        from determined_amd import ops

        ctx.save_for_backward(x, weight)
        y, part = ops.ext().stem_conv_fwd(x, weight, bool(want_stats))
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        from determined_amd import ops

        x, weight = ctx.saved_tensors
        dy = dy.contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:  # images normally need no gradient
            dx = torch.nn.grad.conv2d_input(x.shape, weight.to(dy.dtype), dy, stride=2, padding=3)
        if ctx.needs_input_grad[1]:
            dw = ops.ext().stem_conv_wgrad(x, dy, weight)
        return dx, dw, None


def stem_fusable(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and conv.bias is None and conv.groups == 1
            and conv.in_channels == 3 and conv.out_channels == 64 and conv.kernel_size == (7, 7)
            and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.dilation == (1, 1)
            and conv.padding_mode == "zeros" and conv.weight.dtype in (torch.bfloat16, torch.float32)
            and not x.requires_grad and x.is_contiguous(memory_format=torch.channels_last)):
        return False
    from determined_amd import ops

    return ops.fusion_enabled("stem_conv") and bool(ops.ext().stem_conv_supported(x, conv.weight))


def stem_conv2d(conv: nn.Conv2d, x: torch.Tensor, with_stats: bool = False):
    """``conv(x)`` for the ResNet stem convolution, on the HIP kernels when :func:`stem_fusable`.

    ``with_stats=True`` returns ``(y, part)`` where ``part`` holds the per-channel (sum, sum of
    squares) partials of ``y`` for the following BatchNorm (``BatchNormAct2d.forward_maxpool(...,
    stats_part=part)``) -- or ``None`` when the fallback convolution ran."""
    if stem_fusable(conv, x):
        from determined_amd import ops

        stats = with_stats and ops.fusion_enabled("stem_stats")
        y, part = _StemConvFn.apply(x, conv.weight, stats)
        if not with_stats:
            return y
        return y, (part if stats else None)
    y = conv(x)
    return (y, None) if with_stats else y


class _StemPoolFn(torch.autograd.Function):
    """``maxpool3x3s2p1(relu(bn(conv7x7s2(x))))`` -- the whole ResNet stem -- without the conv's
    full-size output (csrc/conv_stem.hip ``stem_pool_*``): the forward pools the raw conv rows
    on chip by the sign of the BN weight and writes the selected values + window positions; the
    backward recomputes the conv rows and feeds the BN input gradient straight into the weight
    gradient.  Reference: the stem of ``examples/computer_vision`` ResNets (torchvision
    ``resnet50``: conv1 -> bn1 -> relu -> maxpool)."""

    @staticmethod
    def forward(ctx, x, weight, gamma, beta, running_mean, running_var, momentum, eps, split=False):
        from determined_amd import ops

        y, idx, stats, xarg = ops.ext().stem_pool_fwd(x, weight, gamma, beta, running_mean, running_var,
                                                      float(momentum), float(eps))
        ctx.save_for_backward(x, weight, idx, stats, gamma, xarg)
        ctx.set_materialize_grads(False)
        if split:
            return y, y.detach()
        return y

    @staticmethod
    def backward(ctx, dy, dy2=None):
        from determined_amd import ops
        from determined_amd.ops.bn import _sum_grads

        x, weight, idx, stats, gamma, xarg = ctx.saved_tensors
        dy, dy2 = _sum_grads(dy, dy2, torch.channels_last)
        if dy is None:
            return (None,) * 9
        dw, dg, db = ops.ext().stem_pool_bwd(x, weight, dy, dy2, idx, xarg, stats, gamma)
        return None, dw, dg, db, None, None, None, None, None


def stem_bn_pool(conv: nn.Conv2d, bn: nn.Module, pool: nn.MaxPool2d, x: torch.Tensor, split_grad: bool = False):
    """``pool(relu(bn(conv(x))))`` for the ResNet stem: one fused op (:class:`_StemPoolFn`) when
    the conv is :func:`stem_fusable`, ``bn`` a training-mode ``BatchNormAct2d`` with ReLU and
    ``pool`` the 3x3/s2/p1 max-pool; else the stem conv (+ its BN statistics) and
    ``bn.forward_maxpool``.  ``split_grad``: return ``(y, y)`` handles (ops/bn.py)."""
    from determined_amd import ops

    fusable = (stem_fusable(conv, x) and ops.fusion_enabled("stem_pool") and getattr(bn, "act", False)
               and bn.affine and bn.training and bn.track_running_stats and bn.num_batches_tracked is not None
               and pool.kernel_size in (3, (3, 3)) and pool.stride in (2, (2, 2)) and pool.padding in (1, (1, 1))
               and pool.dilation in (1, (1, 1)) and not pool.ceil_mode and not pool.return_indices
               and _plain_module(bn) and _plain_module(pool) and bn.weight.dtype == bn.bias.dtype
               and bn.weight.dtype in (torch.bfloat16, torch.float32) and bool(ops.ext().stem_pool_supported(x, conv.weight)))
    if not fusable:
        y, part = stem_conv2d(conv, x, with_stats=True)
        return bn.forward_maxpool(y, pool, split_grad=split_grad, stats_part=part)
    rm, rv, momentum = bn.train_step_args()
    return _StemPoolFn.apply(x, conv.weight, bn.weight, bn.bias, rm, rv, momentum, bn.eps, split_grad)


def _plain_module(conv: nn.Module) -> bool:
    """No forward hooks / pre-hooks / parametrizations: calling the kernels directly instead of
    ``conv(x)`` would silently skip them."""
    return not (conv._forward_hooks or conv._forward_pre_hooks or hasattr(conv, "parametrizations"))


# ---------------------------------------------------------------------------------------- autotune
# key -> chosen candidate.  Candidates are ints (conv_igemm.hip tile configs) or strings
# ("miopen", "gemm").  DAMD_CONV_TUNE=0 uses the static defaults instead of timing.
_TUNE: Dict[tuple, object] = {}
_TUNE_ON = os.environ.get("DAMD_CONV_TUNE", "1") != "0"


def _parse_exclude(spec: str) -> frozenset:
    """``DAMD_CONV_EXCLUDE="wgrad:8-11,*:14-21"``: candidates removed from the per-layer choice
    (A/B measurements of new kernel configs on one box); ``*`` matches every key kind."""
    out = set()
    for tok in spec.split(","):
        tok = tok.strip()
        if not tok or ":" not in tok:
            continue
        kind, _, cfgs = tok.partition(":")
        lo, _, hi = cfgs.partition("-")
        if not lo.isdigit():
            out.add((kind, cfgs))  # a named candidate ("miopen", "gemm")
            continue
        for c in range(int(lo), int(hi or lo) + 1):
            out.add((kind, c))
    return frozenset(out)


_EXCLUDE = _parse_exclude(os.environ.get("DAMD_CONV_EXCLUDE", ""))
_PRO_ALWAYS_1X1 = os.environ.get("DAMD_PRO_ALWAYS_1X1", "0") == "1"


def _allowed(kind: str, cfg: object) -> bool:
    return (kind, cfg) not in _EXCLUDE and ("*", cfg) not in _EXCLUDE


def exclude_stream_k() -> None:
    """Drop every stream-K tile config from the candidates (and forget choices that picked one):
    called by ``ops.conv_health_check`` after a stream-K hand-off timed out."""
    global _EXCLUDE
    from determined_amd import ops

    e = ops.ext()
    sk = [c for c in range(e.conv_num_cfgs()) if e.conv_sk_cfg(c)]
    _EXCLUDE = _EXCLUDE | frozenset(("*", c) for c in sk)
    for k in [k for k, v in _TUNE.items() if isinstance(v, int) and not isinstance(v, bool) and v in sk]:
        del _TUNE[k]


def _prologue_pays(key: tuple, t_fused: Callable[[], float], t_plain: Callable[[], float]) -> bool:
    """Whether a BN apply fused into a conv's operand staging beats the separate apply pass plus
    the conv's best plain config for this layer (timed once, like the tile choice).  The staging
    is redone for every output-channel tile, so it pays where there are few co tiles and many
    pixels (the 56x56 / 28x28 layers) and loses on the 7x7 layers with 2048 channels (8 co tiles)."""
    global _DB_LOADED
    if not _DB_LOADED:
        _DB_LOADED = True
        load_tune_db()
    if _PRO_ALWAYS_1X1 and len(key) > 2 and len(key[2]) == 4 and key[2][2] == 1:
        return True  # A/B switch: the round-2 behaviour (1x1 prologues never timed)
    got = _TUNE.get(key)
    if got is None:
        got = False
        if _TUNE_ON and not torch.cuda.is_current_stream_capturing():
            global _TUNE_SECONDS
            t0 = time.perf_counter()
            tf, tp = _agreed([t_fused(), t_plain()])
            _TUNE_SECONDS += time.perf_counter() - t0
            got = tf < tp
        _TUNE[key] = got
    return bool(got)


# Multi-rank runs: while set (``agree_across_ranks``), every candidate timing is replaced by its
# mean over the ranks before the choice, so all ranks pick the same kernels (a data-parallel step
# runs at the pace of the slowest rank; independent noisy picks would make some rank slower).
_AGREE: Optional[Callable[[List[float]], List[float]]] = None


def _agreed(times: List[float]) -> List[float]:
    return list(_AGREE(times)) if _AGREE is not None else times


@contextlib.contextmanager
def agree_across_ranks(group=None) -> Iterator[None]:
    """Inside this context the per-layer kernel timings are averaged over the ranks of ``group``
    (a CPU/gloo process group; every rank must run the same layers in the same order, e.g. one
    identical forward/backward per rank).  No-op without an initialised multi-rank group."""
    global _AGREE
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        yield
        return
    world = dist.get_world_size(group)

    def mean(v: List[float]) -> List[float]:
        t = torch.tensor(v, dtype=torch.float64)
        dist.all_reduce(t, group=group)
        return (t / world).tolist()

    prev, _AGREE = _AGREE, mean
    try:
        yield
    finally:
        _AGREE = prev


# Candidate pruning: every candidate is first timed once (after a warm-up call); only those within
# _PRUNE_RATIO of the quickest (at most _PRUNE_KEEP) get the full best-of timing.  Cuts tuning time
# ~2x at large batches (most configs are clearly slower) without changing the choices measurably.
_PRUNE_KEEP = 3
_PRUNE_RATIO = 1.25
_TUNE_SECONDS = 0.0


def tuning_seconds() -> float:
    """Wall seconds spent timing kernel candidates so far (all tuning decisions)."""
    return _TUNE_SECONDS


def _time_quick(fn: Callable[[], object]) -> float:
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e)


def _survivors(quick: Dict[object, float]) -> List[object]:
    best = min(quick.values())
    order = sorted((c for c in quick if quick[c] != float("inf")), key=quick.get)
    return [c for c in order[:_PRUNE_KEEP] if quick[c] <= best * _PRUNE_RATIO] or order[:1]


def _min_time(fns: List[Callable[[], object]]) -> float:
    """Best time over candidate launchers (pruned: full timing only for the near-best)."""
    if len(fns) <= _PRUNE_KEEP:
        return min(_time_once(f) for f in fns)
    quick = {i: _time_quick(f) for i, f in enumerate(fns)}
    return min(_time_once(fns[i]) for i in _survivors(quick))


def _time_once(fn: Callable[[], object], reps: int = 3, rounds: int = 2) -> float:
    """Best of ``rounds`` timings of ``reps`` back-to-back calls (after one warm-up call)."""
    fn()
    best = float("inf")
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        e.synchronize()
        best = min(best, s.elapsed_time(e) / reps)
    return best


# Per-layer choices measured once on an MI355X can be shipped as a file (like MIOpen's find-db):
# DAMD_CONV_TUNE_DB=<path> (e.g. determined_amd/benchmarks/conv_tune_db.jsonl, ResNet-50 at batch
# 512) starts from them -- warm-up 18 s instead of 70 s -- and shapes missing from it are timed as
# before.  Off by default: the headline bench measured ~0.9% faster when the choices are timed in
# the process that runs them (same box, interleaved A/B, profiles/conv_tune_db_ab_1gpu.txt).
_DB_DEFAULT = ""
_DB_LOADED = False


def _tupled(v):
    return tuple(_tupled(x) for x in v) if isinstance(v, list) else v


def load_tune_db(path: Optional[str] = None) -> int:
    """Merge a tuning database (JSON lines ``{"key": [...], "choice": ...}``) into the choices."""
    path = os.environ.get("DAMD_CONV_TUNE_DB", _DB_DEFAULT) if path is None else path
    if not path or not os.path.exists(path):
        return 0
    import json

    n = 0
    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line or line.startswith("#"):
                continue
            rec = json.loads(line)
            _TUNE.setdefault(_tupled(rec["key"]), rec["choice"])
            n += 1
    return n


def save_tune_db(path: str) -> int:
    """Write the choices made so far (for ``load_tune_db``)."""
    import json

    with open(path, "w") as f:
        for k, v in sorted(_TUNE.items(), key=str):
            f.write(json.dumps({"key": k, "choice": v}) + "\n")
    return len(_TUNE)


def _pick(key: tuple, cands: Dict[object, Callable[[], object]], default) -> object:
    global _DB_LOADED
    from determined_amd import ops

    if not _DB_LOADED:
        _DB_LOADED = True
        load_tune_db()
    got = _TUNE.get(key)
    if got is not None and (got in cands or isinstance(got, bool)):
        return got
    if _EXCLUDE:
        kept = {c: f for c, f in cands.items() if (key[0], c) not in _EXCLUDE and ("*", c) not in _EXCLUDE}
        cands = kept or cands
    if not _TUNE_ON or len(cands) <= 1 or torch.cuda.is_current_stream_capturing():
        choice = default if default in cands else next(iter(cands))
    else:
        t_start = time.perf_counter()

        def timed(fn, quick: bool) -> float:
            try:
                return _time_quick(fn) if quick else _time_once(fn)
            except RuntimeError as err:  # a checked launch refused this config (DAMD_LAUNCH): not a candidate
                if "kernel launch failed" not in str(err):
                    raise
                return float("inf")

        pool = list(cands)
        if len(pool) > _PRUNE_KEEP:  # quick pass, agreed across ranks so every rank keeps the same set
            quick = dict(zip(pool, _agreed([timed(cands[c], True) for c in pool])))
            if min(quick.values()) != float("inf"):
                pool = _survivors(quick)
        times = {c: timed(cands[c], False) for c in pool}
        has_sk = any(isinstance(c, int) and ops.ext().conv_sk_cfg(c) for c in cands)
        # one collective per layer carries the candidate times AND the stream-K time-out count, so
        # every rank sees a time-out on any rank and all of them exclude stream-K (and raise) together
        # instead of one rank raising while the others block in the next collective
        n_to = float(ops.conv_sk_timeouts()) if has_sk else 0.0
        agreed = _agreed(list(times.values()) + [n_to])
        times = dict(zip(times, agreed[:-1]))
        if agreed[-1] > 0:
            exclude_stream_k()
            raise RuntimeError(f"stream-K convolution hand-off(s) timed out while tuning {key} (on some rank): the "
                               "affected output tiles were written as NaN; stream-K configs are now excluded")
        choice = min(times, key=times.get)
        global _TUNE_SECONDS
        _TUNE_SECONDS += time.perf_counter() - t_start
        if times[choice] == float("inf"):
            raise RuntimeError(f"no convolution config for {key} launched successfully")
    _TUNE[key] = choice
    return choice


def tuned_choices() -> Dict[tuple, object]:
    """The per-shape kernel choices made so far (for reports / tests)."""
    return dict(_TUNE)


def _igemm_cfgs(ext, x: torch.Tensor, w: torch.Tensor, stride: int, pad: int):
    return [c for c in range(ext.conv_num_cfgs()) if ext.conv_supported(x, w, c, stride, pad)]


def _flip_weight(w: torch.Tensor) -> torch.Tensor:
    """[K, C, R, S] -> [C, K, R, S] rotated by 180 degrees: the stride-1 input gradient is the
    forward convolution of dY with these weights (padding R - 1 - pad).  1x1: the transpose alone
    (one copy kernel instead of a flip kernel + a copy per backward)."""
    if w.shape[2] == 1 and w.shape[3] == 1:
        return w.transpose(0, 1).contiguous(memory_format=torch.channels_last)
    k, c, r, s = w.shape
    if w.is_contiguous(memory_format=torch.channels_last):  # one gather: [K][RS][C] -> [C][RS reversed][K]
        rev = _REV_TAPS.get((r * s, w.device))
        if rev is None:
            rev = _REV_TAPS[(r * s, w.device)] = torch.arange(r * s - 1, -1, -1, device=w.device)
        out = torch.index_select(w.permute(0, 2, 3, 1).reshape(k, r * s, c).permute(2, 1, 0), 1, rev)
        return out.view(c, r, s, k).permute(0, 3, 1, 2)
    return w.flip(2, 3).transpose(0, 1).contiguous(memory_format=torch.channels_last)


_REV_TAPS: Dict[tuple, torch.Tensor] = {}


def _dgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    from determined_amd import ops

    e = ops.ext()

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False,
                                                   [0, 0], 1, [True, False, False])[0]

    k = w.shape[2]
    if stride == 2 and k == 3 and pad == 1 and w.shape[3] == 3 and x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0:
        cands = {"miopen": miopen}
        for c in _phase_cfgs(e, dy, w):
            cands[f"p{c}"] = (lambda c=c: _dgrad_s2_phases(e, dy, w, x.shape, c))
        key = ("dgrad", tuple(dy.shape), tuple(w.shape), stride, pad)
        return cands[_pick(key, cands, default="miopen")]()
    if stride != 1 or 2 * pad != k - 1:
        return miopen()
    wt = _flip_weight(w)
    cands: Dict[object, Callable[[], object]] = {}
    for c in _igemm_cfgs(e, dy, wt, 1, k - 1 - pad):
        cands[c] = (lambda c=c: e.conv_fwd(dy, wt, 1, k - 1 - pad, False, c, 0)[0])
    cands["miopen"] = miopen
    if k == 1:
        n, cout, h, wd = dy.shape
        cin = w.shape[1]

        def gemm():
            d2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            return (d2 @ w.reshape(cout, cin)).view(n, h, wd, cin).permute(0, 3, 1, 2)
        cands["gemm"] = gemm
    key = ("dgrad", tuple(dy.shape), tuple(w.shape), stride, pad)
    return cands[_pick(key, cands, default=next(iter(cands)))]()


# stride-2 3x3 input gradient by phases: dX[2i+a, 2j+b] only sees the taps r with (2i+a+1-r) even --
# a=0: r=1 at dY row i; a=1: r=2 at row i and r=0 at row i+1 (likewise for columns).  Each of the
# four phases is a stride-1 pad-0 conv of dY with a 1x1 / 1x2 / 2x1 / 2x2 sub-kernel whose epilogue
# writes its pixels of dX directly (conv_igemm.hip Geo::ost): 9 taps of MFMA work in all instead of
# the 36 of a zero-inserted dense dgrad, and no zero fill.
_PHASE_TAPS = {0: [1], 1: [2, 0]}  # tap index (r or s) per offset dh = 0, +1


def _phase_weights(w: torch.Tensor):
    ws = []
    for a in (0, 1):
        for b in (0, 1):
            sub = w[:, :, _PHASE_TAPS[a]][:, :, :, _PHASE_TAPS[b]]  # [K][C][Rp][Sp]
            ws.append(((a, b), sub.transpose(0, 1).contiguous(memory_format=torch.channels_last)))
    return ws


def _phase_cfgs(e, dy: torch.Tensor, w: torch.Tensor):
    if not hasattr(e, "conv_dgrad_phase") or dy.dtype != torch.bfloat16 or not dy.is_contiguous(
            memory_format=torch.channels_last):
        return []
    probe = w[:, :, :2, :2].transpose(0, 1).contiguous(memory_format=torch.channels_last)
    return [c for c in range(e.conv_num_cfgs())
            if not e.conv_sk_cfg(c) and e.conv_supported(dy, probe, c, 1, 0) and _allowed("dgrad_phase", c)]


def _dgrad_s2_phases(e, dy: torch.Tensor, w: torch.Tensor, xshape, cfg: int) -> torch.Tensor:
    dx = torch.empty(xshape, device=dy.device, dtype=dy.dtype, memory_format=torch.channels_last)
    for (a, b), sub in _phase_weights(w):
        e.conv_dgrad_phase(dy, sub, dx, a, b, cfg)
    return dx


def _wgrad(dy: torch.Tensor, x: torch.Tensor, w: torch.Tensor, stride: int, pad: int) -> torch.Tensor:
    """Weight gradient: conv_igemm.hip's split-pixel kernel, the 3x3 halo kernels (stride-1 3x3:
    conv_igemm.hip's pixel-run kernel "h0"/"h1", conv3x3v2.hip's whole-row-tile kernels "h2".."h9"), one
    hipBLASLt GEMM for a stride-1 1x1 conv ("gemm") or MIOpen, whichever timed faster for this shape."""
    from determined_amd import ops

    e = ops.ext()

    def miopen():
        return torch.ops.aten.convolution_backward(dy, x, w, None, [stride, stride], [pad, pad], [1, 1], False,
                                                   [0, 0], 1, [False, True, False])[1]

    cands: Dict[object, Callable[[], object]] = {}
    for c in range(e.wgrad_num_cfgs()):
        if e.wgrad_supported(x, dy, w.shape[0], c):
            cands[c] = (lambda c=c: e.conv_wgrad(x, dy, w, stride, pad, c, 0))
    if stride == 1 and pad == 1 and w.shape[2] == 3 and w.shape[3] == 3:  # 3x3 halo kernels
        for c in range(e.wgrad3x3_num_cfgs()):
            if e.wgrad3x3_supported(x, dy, w, c):
                cands[f"h{c}"] = (lambda c=c: e.conv3x3_wgrad(x, dy, w, c, 0))
    if stride in (1, 2) and pad == 0 and w.shape[2] == 1 and w.shape[3] == 1 and x.dtype == dy.dtype:
        # a 1x1 weight gradient is one GEMM over the output pixels, dW[K, C] = dY^T X (hipBLASLt); stride 2
        # takes the even pixels of X (one gathering copy)
        def gemm():
            cout, cin = w.shape[0], w.shape[1]
            d2 = dy.permute(0, 2, 3, 1).reshape(-1, cout)
            xs = x if stride == 1 else x[:, :, ::2, ::2]
            x2 = xs.permute(0, 2, 3, 1).reshape(-1, cin)
            return (d2.t() @ x2).to(w.dtype).view(cout, cin, 1, 1)
        cands["gemm"] = gemm
    cands["miopen"] = miopen
    key = ("wgrad", tuple(x.shape), tuple(w.shape), stride, pad)
    return cands[_pick(key, cands, default="miopen")]()


class _StridedGrad:
    """The input gradient of a 1x1 stride-2 shortcut conv kept on its compact grid.

    A stride-2 1x1 conv reads only the even (h, w) pixels of its input, so its input gradient is
    zero elsewhere: dX[:, :, ::2, ::2] = dY x W^T, a plain stride-1 1x1 input gradient on the
    output grid.  Materialising it at full resolution (MIOpen's strided backward-data + a zero
    fill, then a full-size read by the consumer) moves 4x the bytes.  When the conv's input is
    the ``a`` output of a :class:`_BNActConvFn` node (its only consumer: ``models/resnet.py
    _chain_blocks`` stage transitions), the conv's node returns an unwritten placeholder of the
    input's shape and parks the compact gradient here; that node's backward takes it and adds it
    inside its input-gradient epilogue at the even pixels only (conv_igemm.hip ``EpiArgs.d2h``),
    or materialises it when it cannot fuse."""

    _pending: Dict[int, "_StridedGrad"] = {}

    def __init__(self, placeholder: torch.Tensor, compact: torch.Tensor):
        self.placeholder, self.compact = placeholder, compact

    @classmethod
    def park(cls, x: torch.Tensor, compact: torch.Tensor) -> torch.Tensor:
        ph = torch.empty_like(x, memory_format=torch.channels_last)
        cls._pending[ph.data_ptr()] = cls(ph, compact)
        return ph

    @classmethod
    def take(cls, g: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        if g is None:
            return None
        ent = cls._pending.get(g.data_ptr())
        if ent is None or ent.placeholder.shape != g.shape or ent.placeholder.stride() != g.stride():
            return None
        del cls._pending[g.data_ptr()]
        return ent.compact

    @staticmethod
    def materialise(compact: torch.Tensor, shape) -> torch.Tensor:
        full = torch.zeros(shape, device=compact.device, dtype=compact.dtype).contiguous(
            memory_format=torch.channels_last)
        full[:, :, ::2, ::2] = compact
        return full


def _compact_like(x: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """A shape-only stand-in for a stride-2 1x1 conv's input on its output grid (timing only)."""
    return torch.empty((x.shape[0], x.shape[1]) + tuple(g.shape[2:]), device=x.device, dtype=x.dtype,
                       memory_format=torch.channels_last)


class _IGemmConvFn(torch.autograd.Function):
    """Forward on conv_igemm.hip (+ BN statistic partials); backward: input gradient by
    :func:`_dgrad`, weight gradient by :func:`_wgrad`.  ``compact_dx``: a 1x1 stride-2 conv whose
    input gradient goes to a :class:`_BNActConvFn` node on the compact grid (:class:`_StridedGrad`)."""

    @staticmethod
    def forward(ctx, x, weight, stride, pad, want_stats, cfg, compact_dx=False):
        from determined_amd import ops

        y, part = ops.ext().conv_fwd(x, weight, stride, pad, want_stats, cfg, 0)
        ctx.save_for_backward(x, weight)
        ctx.geo = (stride, pad, bool(compact_dx))
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart=None):
        from determined_amd import ops

        x, weight = ctx.saved_tensors
        stride, pad, compact = ctx.geo
        parked = _LazyBNGrad.take(dy)  # a folded shortcut BN's deferred backward apply (LazyBNResidual)
        dx = dw = None
        if parked is not None:
            e = ops.ext()
            wt = _flip_weight(weight)
            cfgs = ([c for c in range(e.conv_num_cfgs())
                     if e.conv_pro_supported(parked.dz, wt, c) and _allowed("dgrad_pro2", c)]
                    if weight.shape[2] == 1 and weight.shape[3] == 1 and pad == 0 and ctx.needs_input_grad[0] else [])
            if cfgs:  # fused only where it times faster than the apply pass + the plain input gradient
                def t_fused() -> float:
                    return _min_time([lambda c=c: e.conv_fwd_pro2(parked.dz, wt, parked.y, parked.coef, c)
                                      for c in cfgs])

                def t_plain() -> float:
                    g = parked.materialise()
                    return _time_once(parked.materialise) + _time_once(lambda: _dgrad(g, x if stride == 1 else
                                                                                   _compact_like(x, g), weight, 1, 0))

                if not _prologue_pays(("dgrad_pro2_pays", tuple(parked.dz.shape), tuple(weight.shape)), t_fused,
                                      t_plain):
                    cfgs = []
            if cfgs:  # dX with dy = A*dz + B*y + Cc formed in the operand staging; dy returned for dW
                cands = {c: (lambda c=c: e.conv_fwd_pro2(parked.dz, wt, parked.y, parked.coef, c)) for c in cfgs}
                key = ("dgrad_pro2", tuple(parked.dz.shape), tuple(weight.shape))
                dxo, dy = cands[_pick(key, cands, default=cfgs[-1])]()
                if compact:
                    dx = _StridedGrad.park(x, dxo)
                else:  # stride 1: dxo is dX; stride 2 (pad 0): dX is dxo at the even pixels
                    dx = dxo if stride == 1 else _StridedGrad.materialise(dxo, x.shape)
            else:
                dy = parked.materialise()
        dy = dy.contiguous(memory_format=torch.channels_last)
        if ctx.needs_input_grad[0] and dx is None:
            if compact:  # dX on the output grid: the stride-1 1x1 input gradient of dY
                xc = torch.empty((x.shape[0], x.shape[1]) + tuple(dy.shape[2:]), device=x.device, dtype=x.dtype,
                                 memory_format=torch.channels_last)  # shape only (MIOpen candidate)
                dx = _StridedGrad.park(x, _dgrad(dy, xc, weight, 1, 0).contiguous(memory_format=torch.channels_last))
            else:
                dx = _dgrad(dy, x, weight, stride, pad)
        if ctx.needs_input_grad[1]:
            dw = _wgrad(dy, x, weight, stride, pad)
        return dx, dw, None, None, None, None, None


def igemm_fusable(conv: nn.Module, x: torch.Tensor) -> bool:
    if not (isinstance(conv, nn.Conv2d) and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4
            and conv.weight.dtype == torch.bfloat16 and conv.bias is None and conv.groups == 1
            and conv.dilation == (1, 1) and conv.padding_mode == "zeros" and isinstance(conv.padding, tuple)
            and conv.kernel_size[0] == conv.kernel_size[1] and conv.stride[0] == conv.stride[1]
            and conv.padding[0] == conv.padding[1] and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and _plain_module(conv)):
        return False
    from determined_amd import ops

    return ops.fusion_enabled("igemm_conv") and bool(ops.ext().conv_supported(x, conv.weight, -1, conv.stride[0],
                                                                              conv.padding[0]))


def _compact_dx_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """A 1x1 stride-2 conv whose input is the ``a`` output of a :class:`_BNActConvFn` node: its
    input gradient can stay on the compact grid (:class:`_StridedGrad`)."""
    from determined_amd import ops

    return (conv.kernel_size == (1, 1) and conv.stride == (2, 2) and conv.padding == (0, 0) and x.requires_grad
            and isinstance(x.grad_fn, _BNActConvFn._backward_cls) and ops.fusion_enabled("compact_shortcut_grad"))


def conv_bn_input(conv: nn.Conv2d, x: torch.Tensor, stats: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """``(conv(x), stats_part)``: on the implicit-GEMM kernels when :func:`igemm_fusable`,
    ``stats_part`` holding the per-channel (sum, sum of squares) partials of the output for the
    following BatchNorm (``BatchNormAct2d.forward(y, stats_part=part)``); otherwise the module's
    own convolution and ``None``."""
    if not igemm_fusable(conv, x):
        return conv(x), None
    from determined_amd import ops

    e = ops.ext()
    st, pad = conv.stride[0], conv.padding[0]
    w = conv.weight
    key = ("fwd", tuple(x.shape), tuple(w.shape), st, pad)
    cands = {c: (lambda c=c: e.conv_fwd(x, w, st, pad, True, c, 0)) for c in _igemm_cfgs(e, x, w, st, pad)}
    cfg = _pick(key, cands, default=e.conv_default_cfg(w.shape[0]))
    stats = stats and ops.fusion_enabled("conv_stats")
    y, part = _IGemmConvFn.apply(x, w, st, pad, stats, cfg, _compact_dx_ok(conv, x))
    return y, (part if stats else None)


def conv2d(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """``conv(x)`` on the implicit-GEMM kernels where supported (no statistics epilogue)."""
    return conv_bn_input(conv, x, stats=False)[0]


# ------------------------------------------------------------------- BN(+residual)+ReLU -> conv
class _LazyBNGrad:
    """A BatchNorm backward whose apply pass is deferred into the input gradient of the conv that
    produced the BN's input (conv_igemm.hip PRO == 2).  The BN's node returns an unwritten
    placeholder as its input gradient and parks (dz, y, coef) here under the placeholder's
    address; the producing conv's node -- wired to it by ``models/resnet.py _chain_blocks``, the
    only place that sets ``lazy`` -- takes the entry, forms dy = A*dz + B*y + Cc while staging
    its dgrad operand, and gets dy materialised for its weight gradient.  A consumer that cannot
    fuse materialises the entry with the plain apply pass, so the placeholder is never read as
    data."""

    _pending: Dict[int, "_LazyBNGrad"] = {}

    def __init__(self, placeholder: torch.Tensor, dz: torch.Tensor, y: torch.Tensor, coef: torch.Tensor):
        self.placeholder, self.dz, self.y, self.coef = placeholder, dz, y, coef

    @classmethod
    def park(cls, dz: torch.Tensor, y: torch.Tensor, coef: torch.Tensor) -> torch.Tensor:
        ph = torch.empty_like(y)
        cls._pending[ph.data_ptr()] = cls(ph, dz, y, coef)
        return ph

    @classmethod
    def take(cls, g: Optional[torch.Tensor]) -> Optional["_LazyBNGrad"]:
        if g is None:
            return None
        ent = cls._pending.get(g.data_ptr())
        if ent is None or ent.placeholder.shape != g.shape or ent.placeholder.stride() != g.stride():
            return None
        del cls._pending[g.data_ptr()]
        return ent

    def materialise(self) -> torch.Tensor:
        from determined_amd import ops

        return ops.ext().bn_bwd_apply_coef(self.dz, self.y, self.coef)


class LazyBNResidual:
    """A shortcut ``r = bn(y)`` (BatchNorm without ReLU, e.g. ResNet's downsample BN) kept as its
    input ``y`` + the statistic partials of ``y`` from the producing conv.  When the consumer is a
    :func:`bn_act_conv` whose conv stages its operand through the BN prologue, ``r``'s apply pass
    folds into that staging (a = relu(bn(x) + y * r_scale + r_shift); conv_igemm.hip ProArgs
    ``rscale``) and ``r`` is never written; any other consumer calls :meth:`materialise`."""

    def __init__(self, y: torch.Tensor, part: Optional[torch.Tensor], bn: nn.Module, conv: Optional[nn.Module] = None):
        self.y, self.part, self.bn, self.conv = y, part, bn, conv

    def defer_bwd(self) -> bool:
        """Whether this BN's backward apply can move into the producing conv's input gradient:
        ``y`` came out of a 1x1 :class:`_IGemmConvFn` node (its only consumer is the fold)."""
        from determined_amd import ops

        return (self.conv is not None and self.conv.kernel_size == (1, 1) and self.conv.padding == (0, 0)
                and isinstance(self.y.grad_fn, _IGemmConvFn._backward_cls) and ops.fusion_enabled("bn_lazy_bwd"))

    def materialise(self) -> torch.Tensor:
        return self.bn(self.y, stats_part=self.part)


def _materialise(r):
    return r.materialise() if isinstance(r, LazyBNResidual) else r


class _BNActConvFn(torch.autograd.Function):
    """``a = relu(bn(y) [+ residual])``, ``z = conv(a)`` (+ the BN statistic partials of z) as one
    autograd node (the forward apply inside the conv's operand staging where a prologue config
    exists: 1x1 generic tiles, 3x3 halo tiles without a residual), so the backward can fuse the BN's reduce pass into the conv's input-gradient
    epilogue (conv_igemm.hip kEpiBnb*): the gradient at the BN output -- the conv's dX plus the
    gradient ``a`` received from its other consumer (a ResNet shortcut), ReLU-masked -- is
    written once together with its (sum, sum * (y - mean)) partials, and the BN backward is left
    with its finalize and a single apply pass.  That apply pass is itself deferred into the
    producer conv's input gradient when ``lazy`` (:class:`_LazyBNGrad`).  Without the fused kernel
    (strided conv, config unsupported) the backward is the unfused composition."""

    @staticmethod
    def forward(ctx, y, bn_w, bn_b, rm, rv, residual, momentum, eps, stats_part, conv_w, stride, pad, cfg, pro, lazy,
                res_w=None, res_b=None, res_args=None):
        from determined_amd import ops

        e = ops.ext()
        rstats = None
        ctx.res_defer = False
        if res_w is not None:  # residual = bn_r(residual) folded into the prologue (LazyBNResidual)
            r_rm, r_rv, r_mom, r_eps, r_part, ctx.res_defer = res_args
            rstats = e.bn_finalize_part(r_part, residual.numel() // residual.shape[1], res_w, res_b, r_rm, r_rv,
                                        float(r_mom), float(r_eps))
        if pro:  # 1x1 conv applies the BN(+residual)+ReLU while staging its input (conv_igemm.hip PRO)
            stats = e.bn_finalize_part(stats_part, y.numel() // y.shape[1], bn_w, bn_b, rm, rv, float(momentum),
                                       float(eps))
            z, part, a, mask = e.conv_bnact_fwd(y, conv_w, residual, stats, residual is not None, cfg, rstats)
        else:
            a, stats, mask = e.bn_act_fwd(y, bn_w, bn_b, rm, rv, float(momentum), float(eps), residual, True, True,
                                          stats_part)
            z, part = e.conv_fwd(a, conv_w, stride, pad, True, cfg, 0)
        masked = mask.numel() > 0
        ctx.save_for_backward(y, stats, bn_w, mask if masked else None, a, conv_w,
                              residual if (residual is not None and (not masked or rstats is not None)) else None,
                              rstats, res_w)
        ctx.geo = (stride, pad, residual is not None, bool(lazy))
        ctx.mark_non_differentiable(part)
        # an unused `a` (BN1/BN2 outputs have no second consumer) must arrive as None, not as a
        # materialised zero tensor that the backward would read and add
        ctx.set_materialize_grads(False)
        return a, z, part

    @staticmethod
    def backward(ctx, g_a, g_z, _gpart=None):
        from determined_amd import ops

        e = ops.ext()
        y, stats, bn_w, mask, a, conv_w, residual, rstats, res_w = ctx.saved_tensors
        stride, pad, has_res, lazy = ctx.geo
        if rstats is not None:  # the folded residual BN's input is saved, not the residual itself
            res_in, residual = residual, None
        cl = torch.channels_last
        k = conv_w.shape[2]
        if g_z is None:  # the conv output is always consumed in the networks this node serves
            raise RuntimeError("bn_act_conv: the conv output received no gradient")
        g_ac = _StridedGrad.take(g_a)  # a stride-2 shortcut's input gradient on its compact grid
        if g_ac is not None:
            g_a = g_ac
        g_a = None if g_a is None else g_a.contiguous(memory_format=cl)
        parked = _LazyBNGrad.take(g_z)  # g_z may be a deferred BN backward (the next BN's node)
        wt = _flip_weight(conv_w) if stride == 1 and 2 * pad == k - 1 else None
        fused = wt is not None and (mask is not None or not has_res)
        pro_cfgs = ([c for c in range(e.conv_num_cfgs())
                     if e.conv_pro_supported(parked.dz, wt, c) and _allowed("dgrad_bn_pro", c)]
                    if parked is not None and fused else [])
        fused_bwd = None  # (dz, part, dw) from the one-pass 1x1 backward
        if (parked is not None and pro_cfgs and k == 1 and not has_res and mask is None and g_a is None
                and ctx.needs_input_grad[9] and e.conv1x1_bwd_fused_supported(conv_w)
                and _allowed("bwd1x1_fused", 0)):
            dzn, yn, coef = parked.dz, parked.y, parked.coef
            fused_fn = (lambda: e.conv1x1_bwd_fused(dzn, yn, coef, conv_w, a, y, stats))

            def t_fused() -> float:
                return _time_once(fused_fn)

            def t_plain() -> float:
                t_d = _min_time([lambda c=c: e.conv_dgrad_bn(dzn, wt, 0, c, None, y, None, stats, yn, coef)
                                 for c in pro_cfgs])
                gz = e.conv_dgrad_bn(dzn, wt, 0, pro_cfgs[-1], None, y, None, stats, yn, coef)[2]
                return t_d + _time_once(lambda: _wgrad(gz, a, conv_w, 1, 0))

            key = ("bwd1x1_fused_pays", tuple(dzn.shape), tuple(conv_w.shape))
            if _prologue_pays(key, t_fused, t_plain):
                fused_bwd = fused_fn()
                parked = None
        if parked is not None and pro_cfgs and fused_bwd is None:  # 1x1 and 3x3: fused only where it pays
            dzn, yn, coef = parked.dz, parked.y, parked.coef
            plain_cfgs = _igemm_cfgs(e, dzn, wt, 1, k - 1 - pad)

            def t_fused() -> float:
                return _min_time([lambda c=c: e.conv_dgrad_bn(dzn, wt, k - 1 - pad, c, g_a, y, mask, stats, yn,
                                                              coef) for c in pro_cfgs])

            def t_plain() -> float:
                gz = parked.materialise()
                return _time_once(parked.materialise) + _min_time(
                    [lambda c=c: e.conv_dgrad_bn(gz, wt, k - 1 - pad, c, g_a, y, mask, stats, None, None)
                     for c in plain_cfgs])

            key = ("dgrad_pro_pays", tuple(dzn.shape), tuple(conv_w.shape), mask is not None,
                   None if g_a is None else tuple(g_a.shape))
            if not plain_cfgs or not _prologue_pays(key, t_fused, t_plain):
                pro_cfgs = []
        if parked is not None and not pro_cfgs:
            g_z, parked = parked.materialise(), None
        if parked is None and fused_bwd is None:
            g_z = g_z.contiguous(memory_format=cl)
            fused = fused and bool(e.conv_supported(g_z, wt, -1, 1, k - 1 - pad))
        if g_ac is not None and not fused:  # the unfused composition needs it at full size
            g_a = _StridedGrad.materialise(g_a, y.shape)
        if fused:
            if fused_bwd is not None:  # dX (+ BN-backward epilogue) and dW in one pass
                dz, part, _ = fused_bwd
            elif parked is not None:  # BN-backward apply of the next BN inside this dgrad's staging
                dzn, yn, coef = parked.dz, parked.y, parked.coef
                cands = {c: (lambda c=c: e.conv_dgrad_bn(dzn, wt, k - 1 - pad, c, g_a, y, mask, stats, yn, coef))
                         for c in pro_cfgs}
                key = ("dgrad_bn_pro", tuple(dzn.shape), tuple(conv_w.shape), mask is not None,
                       None if g_a is None else tuple(g_a.shape))
                dz, part, g_z = cands[_pick(key, cands, default=pro_cfgs[-1])]()
            else:
                cands = {c: (lambda c=c: e.conv_dgrad_bn(g_z, wt, k - 1 - pad, c, g_a, y, mask, stats, None, None))
                         for c in _igemm_cfgs(e, g_z, wt, 1, k - 1 - pad)}
                key = ("dgrad_bn", tuple(g_z.shape), tuple(conv_w.shape), mask is not None,
                       None if g_a is None else tuple(g_a.shape))
                dz, part = cands[_pick(key, cands, default=e.conv_default_cfg(wt.shape[0]))]()
            if lazy:  # defer this BN's apply pass into the conv that produced y
                coef, dg, db = e.bn_bwd_finalize_part(y, stats, bn_w, part)
                dy = _LazyBNGrad.park(dz, y, coef)
            else:
                dy, dg, db = e.bn_bwd_from_part(dz, y, stats, bn_w, part)
            dres = dz if has_res else None
        else:
            da = _dgrad(g_z, a, conv_w, stride, pad).contiguous(memory_format=cl)
            if g_a is not None and mask is None:
                da, g_a = da + g_a, None
            dy, dg, db, dres = e.bn_act_bwd(da, y, residual, stats, bn_w, True, has_res, mask, g_a)
        if fused_bwd is not None:
            dw = fused_bwd[2]
        else:
            dw = _wgrad(g_z, a, conv_w, stride, pad) if ctx.needs_input_grad[9] else None
        dg_r = db_r = None
        if rstats is not None and dres is not None:  # backward of the folded residual BN (no ReLU)
            dres = dres.contiguous(memory_format=cl)
            if ctx.res_defer:  # its apply pass moves into the shortcut conv's input gradient (PRO 2)
                coef, dg_r, db_r = e.bn_bwd_coef(dres, res_in, rstats, res_w)
                dres = _LazyBNGrad.park(dres, res_in, coef)
            else:
                dres, dg_r, db_r, _ = e.bn_act_bwd(dres, res_in, None, rstats, res_w, False, False, None, None)
        return (dy, dg, db, None, None, dres if has_res else None, None, None, None, dw, None, None, None, None, None,
                dg_r, db_r, None)


def bn_act_conv(bn: nn.Module, y: torch.Tensor, stats_part: Optional[torch.Tensor], residual: Optional[torch.Tensor],
                conv: nn.Conv2d, lazy_grad: bool = False) -> Tuple[torch.Tensor, torch.Tensor, Optional[torch.Tensor]]:
    """``a = bn(y, residual, stats_part=stats_part)`` (a ``BatchNormAct2d`` with ReLU) followed by
    ``z, part = conv_bn_input(conv, a)``; returns ``(a, z, part)``.  Training-mode bf16
    channels-last inputs run as one fused autograd node (:class:`_BNActConvFn`); anything else
    is that exact composition.  ``lazy_grad``: ``y`` is the ``z`` of another ``bn_act_conv``
    node (its only consumer being this one), which may then take this BN's backward apply pass
    into its own input gradient (:class:`_LazyBNGrad`)."""
    from determined_amd import ops
    from determined_amd.ops.bn import BatchNormAct2d

    lres = residual if isinstance(residual, LazyBNResidual) else None
    if lres is not None and not (isinstance(lres.bn, BatchNormAct2d) and not lres.bn.act and _plain_module(lres.bn)
                                 and lres.part is not None and lres.bn.kernel_path(lres.y)
                                 and ops.fusion_enabled("bn_residual_fold")):
        residual, lres = lres.materialise(), None
    rt = lres.y if lres is not None else residual  # the residual operand tensor
    if (isinstance(bn, BatchNormAct2d) and bn.act and _plain_module(bn) and ops.fusion_enabled("bn_conv")
            and igemm_fusable(conv, y) and bn.kernel_path(y, rt) and y.shape[1] == conv.in_channels):
        e = ops.ext()
        rm, rv, momentum = bn.train_step_args()
        st, pad = conv.stride[0], conv.padding[0]
        w = conv.weight
        # Only a producer node that takes the parked entry (_LazyBNGrad.take) may receive the
        # placeholder: if the previous conv fell back to its module (a hook / parametrization on
        # it), its backward would read the unwritten placeholder as dY.
        lazy = (bool(lazy_grad) and ops.fusion_enabled("bn_lazy_bwd") and y.requires_grad
                and isinstance(y.grad_fn, (_BNActConvFn._backward_cls, _IGemmConvFn._backward_cls)))
        pro_cfgs = ([c for c in range(e.conv_num_cfgs()) if e.conv_pro_supported(y, w, c) and _allowed("fwd_pro", c)]
                    if stats_part is not None and ops.fusion_enabled("bn_prologue") and st == 1
                    and 2 * pad == w.shape[2] - 1
                    and (residual is None or w.shape[2] == 1) else [])  # 3x3 prologue: no residual
        if pro_cfgs:  # the fused apply re-stages the operand per co tile: time it against the apply pass
            def t_fused() -> float:  # (only runs when the choice is not cached yet)
                dummy = torch.zeros(4, y.shape[1], device=y.device, dtype=torch.float32)
                dummy[2].fill_(1.0)
                return _min_time([lambda c=c: e.conv_bnact_fwd(y, w, rt, dummy, rt is not None, c, None)
                                  for c in pro_cfgs])

            def t_plain() -> float:
                apply = (lambda: e.bn_act_fwd(y, bn.weight, bn.bias, None, None, 0.0, float(bn.eps), rt, True, True,
                                              stats_part))
                a0 = apply()[0]
                t = _time_once(apply) + _min_time([lambda c=c: e.conv_fwd(a0, w, st, pad, True, c, 0)
                                                   for c in _igemm_cfgs(e, a0, w, st, pad)])
                if lres is not None:  # the plain path also materialises the shortcut BN (no stats update here)
                    t += _time_once(lambda: e.bn_act_fwd(lres.y, lres.bn.weight, lres.bn.bias, None, None, 0.0,
                                                         float(lres.bn.eps), None, False, False, lres.part))
                return t

            if not _prologue_pays(("fwd_pro_pays", tuple(y.shape), tuple(w.shape), rt is not None), t_fused, t_plain):
                pro_cfgs = []
        if lres is not None and not (pro_cfgs and w.shape[2] == 1):  # no 1x1 prologue to fold it into
            residual, lres = lres.materialise(), None
            rt = residual
        if pro_cfgs:  # the BN apply pass moves into the conv's operand staging
            key = ("fwd_pro", tuple(y.shape), tuple(w.shape), rt is not None)
            cfg = _TUNE.get(key)
            if cfg not in pro_cfgs:  # tune on stand-in BN parameters (timing does not depend on them)
                dummy = torch.zeros(4, y.shape[1], device=y.device, dtype=torch.float32)
                dummy[2].fill_(1.0)
                cands = {c: (lambda c=c: e.conv_bnact_fwd(y, w, rt, dummy, rt is not None, c, None))
                         for c in pro_cfgs}
                cfg = _pick(key, cands, default=pro_cfgs[-1])
            if lres is not None:  # the residual's own BN apply folds into the same staging
                r_rm, r_rv, r_mom = lres.bn.train_step_args()
                return _BNActConvFn.apply(y, bn.weight, bn.bias, rm, rv, rt, momentum, bn.eps, stats_part, w, st,
                                          pad, cfg, True, lazy, lres.bn.weight, lres.bn.bias,
                                          (r_rm, r_rv, r_mom, lres.bn.eps, lres.part, lres.defer_bwd()))
            return _BNActConvFn.apply(y, bn.weight, bn.bias, rm, rv, residual, momentum, bn.eps, stats_part, w, st,
                                      pad, cfg, True, lazy)
        key = ("fwd", tuple(y.shape), tuple(w.shape), st, pad)
        cfg = _TUNE.get(key)
        if not isinstance(cfg, int) or not e.conv_supported(y, w, cfg, st, pad):  # tune on a stand-in input
            cands = {c: (lambda c=c: e.conv_fwd(y, w, st, pad, True, c, 0)) for c in _igemm_cfgs(e, y, w, st, pad)}
            cfg = _pick(key, cands, default=e.conv_default_cfg(w.shape[0]))
        return _BNActConvFn.apply(y, bn.weight, bn.bias, rm, rv, residual, momentum, bn.eps, stats_part, w, st, pad,
                                  cfg, False, lazy)
    residual = _materialise(residual)
    a = bn(y, residual, stats_part=stats_part)
    z, part = conv_bn_input(conv, a)
    return a, z, part
