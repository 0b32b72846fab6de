"""Herlev classifier (BASELINE config 4) on the HIP path vs the pinned oracle."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import detgen as G
from oracle import ref_cpu as O
from tests._parity import grad_check, param_keys, perturbed_state

pytestmark = pytest.mark.gpu
K = 7


def herlev_state(stage=4, seed=70):
    spec = O.state_spec(stage, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K)
    return G.make_state(spec, seed)


def build(state, dev, stage=4):
    from ugpg.herlev import HerlevClassificationModel
    m = HerlevClassificationModel(stage, K)
    m.load_state_dict(state)
    return m.to(dev)


def oracle(state, x, y, prev, cw, dtype=torch.float32):
    P = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in state.items()}
    keys = param_keys(P)
    for k in keys:
        P[k].requires_grad_(True)
    out = O.herlev_forward(4, P, x.to(dtype), training=True)
    f, b, w = O.herlev_ug_loss(out, y, None if prev is None else prev.to(dtype), 1.0, K,
                               None if cw is None else cw.to(dtype))
    f.backward()
    return out.detach(), f.detach(), b.detach(), w, {k: P[k].grad for k in keys if P[k].grad is not None}


def test_eval_logits_match_golden(dev):
    fx = np.load("tests/golden/g7_herlev.npz")
    m = build(herlev_state(), dev).eval()
    x = G.randn(71, (4, 3, 64, 64), "x")
    with torch.no_grad():
        out = m(x.to(dev)).cpu()
    assert (out - torch.from_numpy(fx["logits_eval"])).abs().max().item() <= 1e-3


def test_train_step_parity_without_dropout(dev):
    """Train-mode forward (dropout p=0 on both sides, as the golden), UG CE loss with
    the previous stage's logits, gradients vs the fp64 oracle with the perturbation floor."""
    from ugpg.herlev import _CEUGFn
    fx = np.load("tests/golden/g7_herlev.npz")
    state = herlev_state()
    m = build(state, dev).train()
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = G.randn(71, (4, 3, 64, 64), "x")
    y = torch.from_numpy(fx["y"])
    prev = torch.from_numpy(fx["prev_logits"])
    cw = torch.from_numpy(fx["class_weights"])
    out = m(x.to(dev))
    buf = torch.empty(5, device=dev)
    final = _CEUGFn.apply(out, y.to(dev), prev.to(dev), cw.to(dev), 1.0, buf)
    final.backward()
    v = buf.tolist()
    assert (out.detach().cpu() - torch.from_numpy(fx["logits_train"])).abs().max().item() <= 1e-3
    assert abs(v[0] - fx["loss"][0]) <= 1e-5 * abs(fx["loss"][0])
    assert abs(v[1] - fx["loss"][1]) <= 1e-5 * abs(fx["loss"][1])
    w = torch.from_numpy(fx["weights"]).double()
    assert abs(v[2] - w.mean().item()) < 1e-6 and abs(v[3] - w.std().item()) < 1e-5
    assert int(v[4]) == int((out.detach().cpu().argmax(1) == y).sum())
    _, _, _, _, g32 = oracle(state, x, y, prev, cw)
    _, _, _, _, g64 = oracle(state, x, y, prev, cw, torch.float64)
    floor = {k: (g32[k].double() - g64[k]).abs().max().item() for k in g32}
    for s, rel in ((7, 1e-7), (8, 1e-7), (10, 1e-6)):
        _, _, _, _, gp = oracle(perturbed_state(state, s, rel), x, y, prev, cw)
        for k in floor:
            floor[k] = max(floor[k], (gp[k].double() - g64[k]).abs().max().item())
    named = dict(m.named_parameters())
    bad = []
    for k in g32:
        ok, err, bound = grad_check(k, named[k].grad, g32[k], g64[k], floor[k])
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    assert not bad, "\n".join(bad)
    unused = [k for k, p in named.items() if k not in g32]
    assert all(named[k].grad is None for k in unused)  # decoder/head of the wrapped U-Net


def test_dropout_mask_statistics(dev):
    from ugpg import ops
    for p in (0.5, 0.3, 0.2):
        m = ops.dropout_mask(1 << 20, p, 1234, dev).cpu()
        keep = (m > 0).float().mean().item()
        assert abs(keep - (1 - p)) < 3e-3
        assert torch.allclose(m[m > 0], torch.full_like(m[m > 0], 1 / (1 - p)))
        assert torch.equal(m, ops.dropout_mask(1 << 20, p, 1234, dev).cpu())
        assert not torch.equal(m, ops.dropout_mask(1 << 20, p, 1235, dev).cpu())


def test_adam_matches_torch_rule(dev):
    import ugpg.optim as uo
    p0 = G.randn(5, (3000,), "p")
    ref = nn.Parameter(p0.clone())
    ours = nn.Parameter(p0.clone().to(dev))
    topt = torch.optim.Adam([ref], lr=1e-3, weight_decay=1e-4)
    uopt = uo.Adam([ours], lr=1e-3, weight_decay=1e-4)
    for s in range(4):
        g = G.randn(20 + s, (3000,), "g") * 0.1
        ref.grad = g.clone()
        ours.grad = g.to(dev)
        topt.step()
        uopt.step()
    assert (ours.detach().cpu() - ref.detach()).abs().max().item() <= 1e-6
    assert int(uopt.state[ours]["step"]) == 4


def test_trainer_steps_stage4(dev):
    from ugpg.herlev import HerlevTrainer
    tr = HerlevTrainer({"device": dev, "epochs_per_stage": 1, "num_classes": K,
                        "class_weights": [1.0, 1.2, 0.8, 1.5, 1.0, 0.9, 1.1],
                        "stage4_resolution": 64})
    tr.setup_optimizer_scheduler(4)
    x = G.randn(81, (8, 3, 64, 64), "x").to(dev)
    y = G.randint(82, (8,), K, "y").to(dev)
    losses = []
    for _ in range(3):
        out = tr.train_step(x, y, 4)
        losses.append(out.tolist())
    for v in losses:
        assert all(np.isfinite(v[:4])) and 1.0 <= v[2] <= 2.0
    f, metrics = tr.uncertainty_guided_forward_pass(x, y, 4)
    assert set(metrics) == {"final_loss", "base_loss", "output", "uncertainty_weight_mean",
                            "uncertainty_weight_std"}


def _reference_trainer(dev, K, cw, alpha, res4):
    from ugpg.herlev import HerlevTrainer
    return HerlevTrainer({"device": dev, "epochs_per_stage": 1, "num_classes": K,
                          "class_weights": cw, "uncertainty_alpha": alpha, "weight_decay": 1e-4,
                          "stage4_resolution": res4})


def _check_grad_stats(m, fx, rtol=2e-3):
    """Per-tensor gradient norm and sum against the reference's checksums."""
    named = dict(m.named_parameters())
    n = 0
    for key in fx.files:
        if not key.startswith("grad32/"):
            continue
        k = key[len("grad32/"):]
        g = named[k].grad.detach().double().cpu()
        norm, tot = fx[key][0], fx[key][1]
        assert abs(g.norm().item() - norm) <= rtol * norm + 1e-6, (k, g.norm().item(), norm)
        n += 1
    assert n > 0


def test_reference_trainer_step_224(dev):
    """HerlevTrainer.uncertainty_guided_forward_pass at the reference's Stage-4 resolution
    224, bs4, class weights, pinned by the reference trainer itself (G7b)."""
    fx = np.load("tests/golden/g7b_herlev_trainer_step.npz")
    tr = _reference_trainer(dev, K, fx["class_weights"].tolist(), 1.0, 224)
    s4 = G.make_state(O.state_spec(4, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K), 75)
    s3 = G.make_state(O.state_spec(3, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K), 76)
    tr.models[4].load_state_dict(s4)
    tr.models[3].load_state_dict(s3)
    tr.models[4].train()
    for mod in tr.models[4].modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = G.randn(77, (4, 3, 224, 224), "x").to(dev)
    y = G.randint(78, (4,), K, "y").to(dev)
    final, met = tr.uncertainty_guided_forward_pass(x, y, 4)
    final.backward()
    want = fx["loss"]
    got = [met["final_loss"], met["base_loss"], met["uncertainty_weight_mean"],
           met["uncertainty_weight_std"]]
    assert abs(got[0] - want[0]) <= 1e-5 * abs(want[0]) and abs(got[1] - want[1]) <= 1e-5 * abs(want[1])
    assert abs(got[2] - want[2]) <= 1e-5 and abs(got[3] - want[3]) <= 1e-5, (got, want)
    assert (met["output"].detach().cpu() - torch.from_numpy(fx["logits"])).abs().max().item() <= 1e-3
    _check_grad_stats(tr.models[4], fx)


def test_reference_binary_branch(dev):
    """The reference's num_classes <= 2 branch (sigmoid uncertainty, broadcast weights), G7d."""
    fx = np.load("tests/golden/g7d_herlev_binary.npz")
    tr = _reference_trainer(dev, 2, None, 0.7, 64)
    s4 = G.make_state(O.state_spec(4, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, 2), 85)
    s3 = G.make_state(O.state_spec(3, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, 2), 86)
    tr.models[4].load_state_dict(s4)
    tr.models[3].load_state_dict(s3)
    tr.models[4].train()
    for mod in tr.models[4].modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = G.randn(87, (2, 3, 64, 64), "x").to(dev)
    y = G.randint(88, (2,), 2, "y").to(dev)
    final, met = tr.uncertainty_guided_forward_pass(x, y, 4)
    final.backward()
    got = [met["final_loss"], met["base_loss"], met["uncertainty_weight_mean"],
           met["uncertainty_weight_std"]]
    assert np.allclose(got, fx["loss"], rtol=1e-5, atol=1e-6), (got, fx["loss"])
    _check_grad_stats(tr.models[4], fx)


def test_constructor_probe_matches_reference(dev):
    """Constructed with the same seed and moved to the GPU, the model's state equals the
    reference constructor's: initial weights (same RNG draws) and the BatchNorm running
    statistics / num_batches_tracked left by its probe forward (G7c)."""
    from ugpg.herlev import HerlevClassificationModel
    fx = np.load("tests/golden/g7c_herlev_ctor.npz")
    torch.manual_seed(5)
    m = HerlevClassificationModel(stage=4, num_classes=K)
    assert np.array_equal(torch.rand(4).numpy(), fx["rng_after"])
    m = m.to(dev)
    n = 0
    for k, v in m.state_dict().items():
        if f"buf/{k}" in fx.files:
            want = fx[f"buf/{k}"]
            if k.endswith("num_batches_tracked"):
                assert int(v) == int(want), k
            else:
                err = np.abs(v.cpu().numpy() - want).max()
                assert err <= 1e-5 * max(1.0, np.abs(want).max()), (k, err)
            n += 1
    assert n == len([f for f in fx.files if f.startswith("buf/")])


@pytest.mark.parametrize("res", [224, 256])
def test_config4_bs16_parity(dev, res):
    """BASELINE config 4 at its size: Stage-4 Herlev classifier, bs16, 224^2 (the
    reference trainer's Stage-4 resolution) and 256^2, train mode (dropout off), UG CE
    loss with class weights: logits, loss and every gradient vs the fp64 oracle (§8d rule)."""
    from ugpg.herlev import _CEUGFn
    B = 16
    state = herlev_state(seed=90)
    m = build(state, dev).train()
    for mod in m.modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = G.randn(91, (B, 3, res, res), "x")
    y = G.randint(92, (B,), K, "y")
    prev = G.randn(93, (B, K), "prev")
    cw = torch.linspace(0.5, 2.0, K)
    out = m(x.to(dev))
    buf = torch.empty(5, device=dev)
    final = _CEUGFn.apply(out, y.to(dev), prev.to(dev), cw.to(dev), 1.0, buf)
    final.backward()
    o32, f32, _, _, g32 = oracle(state, x, y, prev, cw)
    _, f64, _, _, g64 = oracle(state, x, y, prev, cw, torch.float64)
    assert (out.detach().cpu() - o32).abs().max().item() <= 1e-3
    assert abs(buf[0].item() - f64.item()) <= 1e-5 * abs(f64.item())
    floor = {k: (g32[k].double() - g64[k]).abs().max().item() for k in g32}
    for s, rel in ((7, 1e-7), (10, 1e-6), (12, 5e-6)):
        _, _, _, _, gp = oracle(perturbed_state(state, s, rel), x, y, prev, cw)
        for k in floor:
            floor[k] = max(floor[k], (gp[k].double() - g64[k]).abs().max().item())
    named = dict(m.named_parameters())
    bad, ratios = [], []
    for k in g32:
        ok, err, bound = grad_check(k, named[k].grad, g32[k], g64[k], floor[k])
        ratios.append((err / bound, k))
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    print(f"herlev {res}: gradient headroom (err/bound) worst 3 {sorted(ratios, reverse=True)[:3]}")
    assert not bad, "\n".join(bad)


def _oracle_ug(state4, state3, x, y, cw, dtype=torch.float64):
    """The full UG step of the oracle: prev = the Stage-3 classifier in eval mode on the
    input resized to 128 (train_herlev.py:216-296, oracle.ref_cpu.herlev_train_step)."""
    P3 = {k: (v.clone().to(dtype) if v.is_floating_point() else v.clone()) for k, v in state3.items()}
    with torch.no_grad():
        prev = O.herlev_forward(3, P3, O.resize_bilinear(x.to(dtype), 128), training=False)
    return oracle(state4, x, y, prev, cw, dtype)


@pytest.mark.parametrize("res", [224, 256])
def test_config4_bs16_full_ug_step(dev, res):
    """BASELINE config 4 as the trainer runs it (the bs16 test above feeds random
    `prev` logits): HerlevTrainer.uncertainty_guided_forward_pass at bs16 -- the Stage-3
    classifier's eval prediction on the input resized to 128, the uncertainty-weighted CE
    with class weights, backward -- against the oracle's same step (prev from its own
    Stage-3 forward), dropout off: loss, U statistics and every gradient (§8d rule)."""
    B = 16
    cw = [0.5, 0.75, 1.0, 1.25, 1.5, 1.75, 2.0]
    tr = _reference_trainer(dev, K, cw, 1.0, res)
    s4, s3 = herlev_state(4, seed=94), herlev_state(3, seed=95)
    tr.models[4].load_state_dict(s4)
    tr.models[3].load_state_dict(s3)
    tr.models[4].train()
    for mod in tr.models[4].modules():
        if isinstance(mod, nn.Dropout):
            mod.p = 0.0
    x = G.randn(96, (B, 3, res, res), "x")
    y = G.randint(97, (B,), K, "y")
    final, met = tr.uncertainty_guided_forward_pass(x.to(dev), y.to(dev), 4)
    final.backward()
    cwt = torch.tensor(cw)
    o32, f32, b32, w32, g32 = _oracle_ug(s4, s3, x, y, cwt, torch.float32)
    _, f64, b64, w64, g64 = _oracle_ug(s4, s3, x, y, cwt, torch.float64)
    assert (met["output"].detach().cpu() - o32).abs().max().item() <= 1e-3
    assert abs(met["final_loss"] - f64.item()) <= 1e-5 * abs(f64.item())
    assert abs(met["base_loss"] - b64.item()) <= 1e-5 * abs(b64.item())
    assert abs(met["uncertainty_weight_mean"] - w64.mean().item()) <= 1e-5
    floor = {k: (g32[k].double() - g64[k]).abs().max().item() for k in g32}
    for sd, rel in ((7, 1e-7), (10, 1e-6), (12, 5e-6)):
        _, _, _, _, gp = _oracle_ug(perturbed_state(s4, sd, rel), s3, x, y, cwt, torch.float32)
        for k in floor:
            floor[k] = max(floor[k], (gp[k].double() - g64[k]).abs().max().item())
    named = dict(tr.models[4].named_parameters())
    bad, ratios = [], []
    for k in g32:
        ok, err, bound = grad_check(k, named[k].grad, g32[k], g64[k], floor[k])
        ratios.append((err / bound, k))
        if not ok:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    print(f"herlev UG {res}: gradient headroom (err/bound) worst 3 {sorted(ratios, reverse=True)[:3]}")
    assert not bad, "\n".join(bad)
