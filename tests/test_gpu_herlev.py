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
