"""Numerics of the native NHWC conv / BN kernels (csrc/conv.hip, csrc/bn.hip) against PyTorch fp32
references of the same ops on the same bf16-rounded inputs."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

# (N, C, H, W, Cout, R, stride, pad)
SHAPES = [
    (2, 16, 16, 16, 32, 3, 1, 1),
    (2, 64, 14, 14, 128, 3, 2, 1),
    (2, 64, 8, 8, 256, 1, 1, 0),
    (2, 256, 8, 8, 512, 1, 2, 0),
    (2, 3, 32, 32, 64, 7, 2, 3),     # image stem: channels padded to 8
    (1, 24, 9, 7, 40, 3, 1, 1),      # ragged everything
    (4, 64, 56, 56, 64, 3, 1, 1),    # many pixel tiles
    # stride-2 data gradients run as 4 output-parity classes: odd extents give unequal classes
    (1, 24, 9, 7, 40, 3, 2, 1),
    (2, 16, 7, 7, 32, 1, 2, 0),      # 1x1 stride 2: three classes have no tap (zeros)
    # grids far below the CU count with long K loops run split-K (ordered slice sum + epilogue)
    (2, 512, 7, 7, 512, 3, 1, 1),    # forward and data gradient split 4
    (2, 1024, 7, 7, 256, 1, 1, 0),   # forward split 2
]


def _rel(a, b):
    return float((a.float() - b.float()).norm() / (b.float().norm() + 1e-12))


def _inputs(N, C, H, W, Cout, R, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn(N, C, H, W, device="cuda", generator=g).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last)
    w = (torch.randn(Cout, C, R, R, device="cuda", generator=g) * (2.0 / (C * R * R)) ** 0.5).to(torch.bfloat16)
    return x, w


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_forward_and_stats(shape):
    from trustworthy_dl.ops.conv import _Conv2dNHWC
    N, C, H, W, Cout, R, st, pad = shape
    x, w = _inputs(N, C, H, W, Cout, R)
    y, stats = _Conv2dNHWC.apply(x, w, st, pad, True)
    ref = F.conv2d(x.float(), w.float(), None, st, pad)
    assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
    assert _rel(y, ref) < 1e-2
    yb = y.float()
    assert _rel(stats[:Cout], yb.sum((0, 2, 3))) < 1e-3
    assert _rel(stats[Cout:], (yb * yb).sum((0, 2, 3))) < 1e-3


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_backward(shape):
    from trustworthy_dl.ops.conv import conv2d
    N, C, H, W, Cout, R, st, pad = shape
    x, w = _inputs(N, C, H, W, Cout, R, seed=1)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    ref = F.conv2d(xr, wr, None, st, pad)
    gy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16)
    ref.backward(gy.float())
    xn, wn = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = conv2d(xn, wn, st, pad)
    y.backward(gy.contiguous(memory_format=torch.channels_last))
    assert _rel(xn.grad, xr.grad) < 1e-2
    assert _rel(wn.grad, wr.grad) < 1e-2


def test_conv_wgrad_accumulates_into_main_grad():
    from trustworthy_dl.ops.conv import conv2d
    x, w = _inputs(2, 32, 12, 12, 64, 3, seed=2)
    w = w.clone().requires_grad_(True)
    w.main_grad = torch.full(w.shape, 0.5, dtype=torch.float32, device="cuda")
    gy = torch.randn(2, 64, 12, 12, device="cuda").to(torch.bfloat16)
    for _ in range(2):
        conv2d(x, w, 1, 1).backward(gy)
    assert w.grad is None
    wr = w.detach().float().requires_grad_(True)
    F.conv2d(x.float(), wr, None, 1, 1).backward(gy.float())
    assert _rel(w.main_grad - 0.5, 2 * wr.grad) < 1e-2


@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
def test_conv_bn_act_train_matches_torch(relu, residual):
    from trustworthy_dl.ops.conv import conv_bn_act
    torch.manual_seed(0)
    conv = nn.Conv2d(32, 64, 3, 2, 1, bias=False).cuda()
    bn = nn.BatchNorm2d(64).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    conv_r, bn_r = nn.Conv2d(32, 64, 3, 2, 1, bias=False).cuda(), nn.BatchNorm2d(64).cuda()
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    conv.to(torch.bfloat16)
    bn.weight.data = bn.weight.data.to(torch.bfloat16)
    bn.bias.data = bn.bias.data.to(torch.bfloat16)
    conv_r.weight.data.copy_(conv.weight.data.float())
    bn_r.weight.data.copy_(bn.weight.data.float())
    bn_r.bias.data.copy_(bn.bias.data.float())

    x = torch.randn(4, 32, 16, 16, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn(4, 64, 8, 8, device="cuda").to(torch.bfloat16) if residual else None
    xn = x.clone().requires_grad_(True)
    rn = res.clone().requires_grad_(True) if residual else None
    out = conv_bn_act(xn, conv, bn, relu=relu, residual=rn)
    xr = x.float().requires_grad_(True)
    rr = res.float().requires_grad_(True) if residual else None
    ref = bn_r(conv_r(xr))
    if residual:
        ref = ref + rr
    if relu:
        # the ReLU mask of the bf16 output decides near-zero pre-activations; use the same mask in
        # the fp32 reference so mask flips at |pre| ~ bf16 ulp do not masquerade as kernel error
        assert _rel(out, F.relu(ref)) < 2e-2
        ref = ref * (out.detach() > 0).float()
    assert _rel(out, ref) < 2e-2
    gy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16)
    out.backward(gy)
    ref.backward(gy.float())
    assert _rel(xn.grad, xr.grad) < 3e-2
    assert _rel(conv.weight.grad, conv_r.weight.grad) < 3e-2
    assert _rel(bn.weight.grad, bn_r.weight.grad) < 3e-2
    assert _rel(bn.bias.grad, bn_r.bias.grad) < 3e-2
    if residual:
        assert _rel(rn.grad, rr.grad) < 2e-2
    assert _rel(bn.running_mean, bn_r.running_mean) < 2e-2
    assert _rel(bn.running_var, bn_r.running_var) < 2e-2


@pytest.mark.parametrize("n,cin,cout,hw", [(64, 64, 2048, 7), (8, 64, 4096, 7), (16, 16, 64, 112)])
def test_bn_act_production_shapes_match_fp32(n, cin, cout, hw):
    """BN(+residual+ReLU) forward / backward at ResNet-50 stored-output BN shapes and beyond: C = 2048
    (one channel-vector block), C = 4096 (two), and 200k rows at C = 64 (the most row chunks) —
    the atomic-free backward reduction (partial rows + grouped fold) against an fp32 reference."""
    from trustworthy_dl.ops.conv import conv_bn_act
    torch.manual_seed(1)
    conv = nn.Conv2d(cin, cout, 1, 1, 0, bias=False).cuda()
    bn = nn.BatchNorm2d(cout).cuda()
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    conv_r, bn_r = nn.Conv2d(cin, cout, 1, 1, 0, bias=False).cuda(), nn.BatchNorm2d(cout).cuda()
    conv_r.load_state_dict(conv.state_dict())
    bn_r.load_state_dict(bn.state_dict())
    conv.to(torch.bfloat16)
    bn.weight.data = bn.weight.data.to(torch.bfloat16)
    bn.bias.data = bn.bias.data.to(torch.bfloat16)
    conv_r.weight.data.copy_(conv.weight.data.float())
    bn_r.weight.data.copy_(bn.weight.data.float())
    bn_r.bias.data.copy_(bn.bias.data.float())
    x = torch.randn(n, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn(n, cout, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    xn, rn = x.clone().requires_grad_(True), res.clone().requires_grad_(True)
    out = conv_bn_act(xn, conv, bn, relu=True, residual=rn)
    xr, rr = x.float().requires_grad_(True), res.float().requires_grad_(True)
    ref = bn_r(conv_r(xr)) + rr
    assert _rel(out, F.relu(ref)) < 2e-2
    ref = ref * (out.detach() > 0).float()
    gy = torch.randn(ref.shape, device="cuda").to(torch.bfloat16)
    out.backward(gy)
    ref.backward(gy.float())
    assert _rel(xn.grad, xr.grad) < 3e-2
    assert _rel(rn.grad, rr.grad) < 2e-2
    assert _rel(bn.weight.grad, bn_r.weight.grad) < 3e-2
    assert _rel(bn.bias.grad, bn_r.bias.grad) < 3e-2


def _chain_modules(cin, mid, cout, stride, seed):
    torch.manual_seed(seed)
    units = [(nn.Conv2d(cin, mid, 1, 1, 0, bias=False), nn.BatchNorm2d(mid)),
             (nn.Conv2d(mid, mid, 3, stride, 1, bias=False), nn.BatchNorm2d(mid)),
             (nn.Conv2d(mid, cout, 1, 1, 0, bias=False), nn.BatchNorm2d(cout))]
    for _, bn in units:
        with torch.no_grad():
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.uniform_(-0.3, 0.3)
    return units


@pytest.mark.parametrize("stride,widths,hw", [(1, (64, 32, 64), 16), (2, (64, 32, 64), 16),
                                              (1, (256, 128, 256), 8)])   # last: conv2 fwd / dgrad split-K
def test_bn_fold_chain_matches_unfolded_and_fp32(stride, widths, hw, monkeypatch):
    """Bottleneck chain conv1-BN1-ReLU-conv2-BN2-ReLU-conv3-BN3(+res)-ReLU with BN1/BN2 + ReLU folded
    into conv2 / conv3 (tdl_bn_finalize + tdl_conv_nt_pro / tdl_conv_wgrad_pro + tdl_bn_act_bwd_pro:
    the BN outputs are never written) against the unfolded native path and an fp32 torch reference:
    output, input / residual / weight / BN gradients and running statistics."""
    from trustworthy_dl.ops import conv as conv_mod
    from trustworthy_dl.ops.conv import conv_bn_chain
    folded = []
    orig = conv_mod._BNActConvNHWC.apply
    monkeypatch.setattr(conv_mod._BNActConvNHWC, "apply", lambda *a: folded.append(1) or orig(*a))
    cin, mid, cout = widths
    x = torch.randn(4, cin, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = torch.randn(4, cout, hw // stride, hw // stride, device="cuda").to(torch.bfloat16)
    gy = torch.randn(4, cout, hw // stride, hw // stride, device="cuda").to(torch.bfloat16)
    runs = {}
    for fold in ("1", "0"):
        monkeypatch.setenv("TDL_BN_FOLD", fold)
        units = _chain_modules(cin, mid, cout, stride, 0)
        for conv, bn in units:
            conv.cuda().to(torch.bfloat16)
            bn.cuda()
            bn.weight.data = bn.weight.data.to(torch.bfloat16)
            bn.bias.data = bn.bias.data.to(torch.bfloat16)
        xn, rn = x.clone().requires_grad_(True), res.clone().requires_grad_(True)
        n0 = len(folded)
        out = conv_bn_chain(xn, units, relu=True, residual=rn)
        assert len(folded) - n0 == (2 if fold == "1" else 0)   # BN1 / BN2 folded only when enabled
        out.backward(gy)
        runs[fold] = (out.detach().float(), xn.grad.float(), rn.grad.float(),
                      [c.weight.grad.float() for c, _ in units], [b.weight.grad.float() for _, b in units],
                      [b.bias.grad.float() for _, b in units], [b.running_mean.clone() for _, b in units],
                      [b.running_var.clone() for _, b in units])
    # fp32 reference with the same (bf16-rounded) parameters
    units_r = _chain_modules(cin, mid, cout, stride, 0)
    for conv, bn in units_r:
        conv.cuda()
        bn.cuda()
        conv.weight.data = conv.weight.data.to(torch.bfloat16).float()
        bn.weight.data = bn.weight.data.to(torch.bfloat16).float()
        bn.bias.data = bn.bias.data.to(torch.bfloat16).float()
    xr, rr = x.float().requires_grad_(True), res.float().requires_grad_(True)
    h = xr
    for i, (conv, bn) in enumerate(units_r):
        h = bn(conv(h))
        h = F.relu(h + rr) if i == 2 else F.relu(h)
    h.backward(gy.float())
    # folded vs unfolded native: the same per-channel fold and bf16 rounding (bit-identical on
    # MI355X); vs fp32 torch: bf16 error of a 3-conv / 3-BN chain incl. ReLU-mask flips at
    # |pre| ~ 1 ulp (input gradient ~7 %, residual gradient ~5 %)
    f, u = runs["1"], runs["0"]
    assert _rel(f[0], u[0]) < 1e-2 and _rel(f[0], h.detach()) < 5e-2
    assert _rel(f[1], u[1]) < 1e-2 and _rel(f[1], xr.grad) < 1e-1
    assert _rel(f[2], u[2]) < 1e-2 and _rel(f[2], rr.grad) < 1e-1
    for i in range(3):
        assert _rel(f[3][i], u[3][i]) < 1e-2 and _rel(f[3][i], units_r[i][0].weight.grad) < 1e-1, i
        assert _rel(f[4][i], u[4][i]) < 1e-2 and _rel(f[4][i], units_r[i][1].weight.grad) < 1e-1, i
        assert _rel(f[5][i], u[5][i]) < 1e-2 and _rel(f[5][i], units_r[i][1].bias.grad) < 1e-1, i
        assert _rel(f[6][i], units_r[i][1].running_mean) < 2e-2 and _rel(f[7][i], units_r[i][1].running_var) < 2e-2


def test_resnet_engine_step_native():
    """A ResNet-32 pipeline step on the GPU goes through the native conv path (bf16) and matches
    the CPU fp32 engine's first loss."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    g = torch.Generator().manual_seed(3)
    batch = {"input": torch.randn(16, 3, 32, 32, generator=g), "target": torch.randint(0, 10, (16,), generator=g)}
    losses = {}
    for dev in ("cpu", "cuda:0"):
        m = get_model("resnet32", seed=5)
        eng = PipelineEngine(m, EngineConfig(num_nodes=2, micro_batches=2, device=dev,
                                             adamw=AdamWConfig(lr=1e-3), reassign=False))
        eng.train_step(batch)
        eng.train_step(batch)
        eng.flush()
        losses[dev] = eng.last_loss
        if dev.startswith("cuda"):
            assert eng.dtype == torch.bfloat16
    assert losses["cuda:0"] == pytest.approx(losses["cpu"], rel=5e-2)


def test_vgg16_224_gpu_matches_cpu_fp32():
    """VGG-16 (BN) at ImageNet shape, incl. the 25088->4096->4096->1000 classifier: the GPU bf16
    engine (native conv kernels) follows the CPU fp32 engine step by step and the loss stays sane
    (the r1 bench's loss of 99 was AdamW lr 1e-3 diverging on CPU fp32 as well:
    profiles/r2_vgg16_lr_cpu_fp32.json)."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.flat import AdamWConfig
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    from trustworthy_dl.utils.metrics import MetricsCollector
    g = torch.Generator().manual_seed(0)
    batches = [{"input": torch.randn(4, 3, 224, 224, generator=g), "target": torch.randint(0, 1000, (4,), generator=g)}
               for _ in range(2)]
    traj = {}
    for dev in ("cpu", "cuda:0"):
        m = get_model("vgg16", num_classes=1000, image_size=224, seed=1)
        eng = PipelineEngine(m, EngineConfig(num_nodes=1, micro_batches=1, device=dev, reassign=False,
                                             adamw=AdamWConfig(lr=1e-4, weight_decay=1e-4, max_grad_norm=1.0)),
                             metrics=MetricsCollector())
        for i in range(3):
            eng.train_step(batches[i % 2])
        eng.flush()
        traj[dev] = [r["loss"] for r in eng.metrics.batch_metrics]
    cpu, gpu = traj["cpu"], traj["cuda:0"]
    assert gpu[0] == pytest.approx(cpu[0], rel=2e-2)       # same forward at init
    assert gpu[1] == pytest.approx(cpu[1], rel=1e-1)       # same first update
    assert all(l < 9.0 for l in gpu), gpu                   # no divergence (ln 1000 = 6.9)
    assert gpu[-1] < gpu[0]


@pytest.mark.parametrize("k,stride,pad,shape", [(3, 2, 1, (4, 64, 56, 56)), (3, 2, 1, (2, 16, 15, 13)),
                                                (2, 2, 0, (2, 64, 32, 32)), (2, 2, 0, (1, 8, 7, 9))])
def test_max_pool_nhwc_matches_torch(k, stride, pad, shape):
    """Native NHWC max-pool forward / backward vs fp32 torch (small-integer inputs, exact in bf16;
    ties go to the first window position in row-major order in both)."""
    from trustworthy_dl.ops import max_pool2d
    torch.manual_seed(0)
    N, C, H, W = shape
    base = (torch.randperm(N * C * H * W) % 251).float().reshape(shape) - 125.0
    x = base.bfloat16().to("cuda").contiguous(memory_format=torch.channels_last)
    x = x.requires_grad_(True)
    y = max_pool2d(x, k, stride, pad)
    g = torch.randn(y.shape, device="cuda").bfloat16()
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    yr = torch.nn.functional.max_pool2d(xr, k, stride, pad)
    yr.backward(g.float())
    assert torch.equal(y.float(), yr)
    assert float((x.grad.float() - xr.grad).abs().max()) <= 2e-2 * float(xr.grad.abs().max())


@pytest.mark.parametrize("shape", [(4, 2048, 7, 7), (3, 64, 5, 3)])
def test_global_avg_pool_nhwc_matches_torch(shape):
    from trustworthy_dl.ops import global_avg_pool
    torch.manual_seed(1)
    x = torch.randn(shape, device="cuda").bfloat16().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = global_avg_pool(x)
    g = torch.randn(y.shape, device="cuda").bfloat16()
    y.backward(g)
    xr = x.detach().float().requires_grad_(True)
    yr = torch.nn.functional.adaptive_avg_pool2d(xr, 1).flatten(1)
    yr.backward(g.float())
    assert _rel(y, yr) < 1e-2
    assert _rel(x.grad, xr.grad) < 1e-2


def test_resnet50_stage_fwd_bwd_bitwise_repeatable():
    """The recompute audit evaluates a stage twice and compares: the native conv / BN path must be
    bitwise repeatable (BatchNorm statistics and backward sums reduced in a fixed order, no float
    atomics in their order-sensitive folds).  Two forward + backward evaluations of ResNet-50's first
    two pipeline stages on the same inputs and weights: identical outputs and input gradients; the
    weight-gradient sketches agree to fp32 rounding (split-K weight gradients still add their fp32
    slices with atomics: order-dependent in the last bits only, nothing downstream amplifies them)."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    m = get_model("resnet50", num_classes=1000, seed=1)
    eng = PipelineEngine(m, EngineConfig(num_nodes=4, micro_batches=1, device="cuda:0", reassign=False))
    st0, st1 = eng.stages[eng.plan.ranks[0]], eng.stages[eng.plan.ranks[1]]
    x0 = eng._stage_input(torch.randn(8, 3, 224, 224, generator=torch.Generator().manual_seed(0)), st0)
    gy = torch.Generator(device="cuda").manual_seed(1)
    with torch.no_grad():
        y0, _ = st0.forward(x0, None)
        y1, _ = st1.forward(y0, None)
    dy0 = torch.randn(y0.shape, device=y0.device, generator=gy).to(y0.dtype)
    dy1 = torch.randn(y1.shape, device=y1.device, generator=gy).to(y1.dtype)
    runs = [eng._recompute(st0, x0, dy0, None, 1, backward=True) + eng._recompute(st1, y0, dy1, None, 1, backward=True)
            for _ in range(2)]
    for i, (a, b) in enumerate(zip(*runs)):
        if a is None:
            continue
        if i % 3 == 2:    # weight-gradient sketch
            assert float((a - b).abs().max() / b.abs().max()) < 1e-5, i
        else:
            assert torch.equal(a, b), i


def test_resnet50_backward_audit_clean_on_gpu():
    """A clean local ResNet-50 run with the forward + backward audit on (8 stages, micro-batch 8):
    no stage is blamed (round 4's first GPU run blamed every stage: order-dependent float atomics
    in the BN reductions made the recompute differ)."""
    from trustworthy_dl.models import get_model
    from trustworthy_dl.parallel.pipeline import EngineConfig, PipelineEngine
    m = get_model("resnet50", num_classes=1000, seed=1)
    eng = PipelineEngine(m, EngineConfig(num_nodes=8, micro_batches=4, device="cuda:0", monitor_seed=0,
                                         reassign=False))
    g = torch.Generator().manual_seed(0)
    for _ in range(3):
        eng.train_step({"input": torch.randn(32, 3, 224, 224, generator=g),
                        "target": torch.randint(0, 1000, (32,), generator=g)})
    eng.flush()
    assert eng.attack_history == []


def test_batched_weight_layouts_match_permutes():
    """prebuild_layouts (one LDS-tiled launch for many weights, tiles spread by size) writes the same
    [Cout][R][S][Cp] / [Cp][R][S][Cout] images as the per-weight path, padded channels zero."""
    from trustworthy_dl.ops.conv import _weight_layout, prebuild_layouts
    from trustworthy_dl.ops import layers
    shapes = [(64, 3, 7, 7), (512, 512, 3, 3), (40, 24, 3, 3), (2048, 512, 1, 1), (72, 200, 1, 1), (8, 8, 3, 3)]
    ws = [torch.randn(s, device="cuda").to(torch.bfloat16) for s in shapes]
    layers._WEIGHT_GEN[0] += 1
    prebuild_layouts(ws)
    for w in ws:
        Cout, C, R, S = w.shape
        cp = (C + 7) // 8 * 8
        wp = torch.zeros((Cout, cp, R, S), dtype=w.dtype, device=w.device)
        wp[:, :C] = w
        assert torch.equal(_weight_layout(w, cp, "krsc"), wp.permute(0, 2, 3, 1).contiguous())
        assert torch.equal(_weight_layout(w, cp, "crsk"), wp.permute(1, 2, 3, 0).contiguous())
