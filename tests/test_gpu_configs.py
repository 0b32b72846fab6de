"""Parity at the configurations BASELINE.json names, at their stated size.

Config 2 (the benchmarked workload): PGUNet4 uncertainty-guided step at bs16 x 256^2 --
S3@128 eval U map, weighted BCE (pos_weight 5), backward, RMSprop -- checked against the
reference's own bs16 checksums (golden G4b: loss, per-sample logit sums, U statistics,
BN buffers, post-step parameters) and against the fp64 oracle tensor by tensor with the
§8d rule and the reference's measured fp32 noise floors (committed in G4b).  The persistent
conv kernels' work split and the split-K weight-gradient plans depend on the batch size,
so this is the only test that exercises the benchmarked launch shapes.  Under bf16
arithmetic (config 3's) the same step is compared with the oracle run in bf16."""
import numpy as np
import pytest
import torch
import torch.nn as nn

from oracle import detgen as G
from oracle import ref_cpu as O
from tests._parity import det_state, grad_check, is_prebn_bias, oracle_run, param_keys

pytestmark = pytest.mark.gpu


def _inputs():
    from oracle.make_goldens import G4B as c
    state = det_state(4, 3, 1, seed=c["w_seed"])
    prev = det_state(3, 3, 1, seed=c["prev_seed"])
    x = G.randn(c["x_seed"], (c["B"], 3, c["res"], c["res"]), "x")
    t = G.bernoulli(c["t_seed"], (c["B"], 1, c["res"], c["res"]), 0.5, "t")
    return state, prev, x, t


def _hip_step(dev, state, prev, x, t):
    import ugpg
    m = ugpg.PGUNet4(3, 1)
    m.load_state_dict(state)
    m = m.to(dev).train()
    mp = ugpg.PGUNet3(3, 1)
    mp.load_state_dict(prev)
    mp = mp.to(dev)
    L = ugpg.UncertaintyGuidedLoss(dev)
    xd, td = x.to(dev), t.to(dev)
    u = L.generate_uncertainty_map(xd, mp, 128, 256)
    out = m(xd)
    crit = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([5.0], device=dev), reduction="none")
    final, base = L.apply_uncertainty_weighted_loss(crit, out, td, u, 1.0)
    lg_fwd = out.detach().clone()
    final.backward()
    # the backward must leave the forward's logits alone
    assert torch.equal(out.detach(), lg_fwd), "the backward pass modified the forward's logits"
    grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
    opt = ugpg.RMSprop(m.parameters(), lr=1e-4, weight_decay=1e-4)
    opt.step()
    torch.cuda.synchronize()
    return m, out.detach().cpu(), u.cpu(), final.item(), base, grads


# Gradients of config 2 that miss SURVEY §8d's literal rule (2x the reference's UNPERTURBED
# fp32 error + 1e-6 of scale), each one where the reference's own fp32 runs under ulp-level
# weight perturbations (G4b floor_pert) exceed that literal bound too -- checked per tensor
# below and listed with the numbers in DESIGN §4.
LITERAL_RULE_EXCEPTIONS = (
    "inc.conv.conv_op.1.bias", "down2.mpconv.1.conv_op.3.weight",
    "down4.mpconv.1.conv_op.3.weight", "down4.mpconv.1.conv_op.4.weight",
    "down4.mpconv.1.conv_op.4.bias", "up1.conv.conv_op.1.weight", "up1.conv.conv_op.4.bias",
    "up2.conv.conv_op.1.weight", "up2.conv.conv_op.4.bias", "up3.conv.conv_op.1.bias")


def test_config2_bs16_step_parity(dev):
    fx = np.load("tests/golden/g4b_pgunet4_bs16.npz")
    state, prev, x, t = _inputs()
    m, logits, u, final, base, grads = _hip_step(dev, state, prev, x, t)
    # against the reference's own bs16 checksums
    assert abs(final - fx["loss"][2]) <= 1e-5 * abs(fx["loss"][2]), (final, fx["loss"])
    assert abs(base - fx["loss"][1]) <= 1e-5 * abs(fx["loss"][1])
    assert abs(u.mean().item() - fx["u_stats"][0]) <= 1e-5 and abs(u.std().item() - fx["u_stats"][1]) <= 1e-5
    sums = logits.double().sum(dim=(1, 2, 3)).numpy()
    assert np.abs(sums - fx["logits_sample_sums"]).max() <= 1e-3 * 65536 ** 0.5, sums - fx["logits_sample_sums"]
    pred = O.predictions(logits)
    dice = O.dice(pred, t.squeeze(1)).item()
    assert abs(dice - fx["dice_acc"][0]) <= 1e-3 and abs(O.accuracy(pred, t.squeeze(1).long()) - fx["dice_acc"][1]) <= 1e-3
    sd = m.state_dict()
    for k, v in sd.items():
        key = f"buf/{k}"
        if key in fx.files:
            want = fx[key]
            if k.endswith("num_batches_tracked"):
                assert int(v) == int(want), k
            else:
                assert np.abs(v.cpu().numpy() - want).max() <= 1e-5 * max(1.0, np.abs(want).max()), k
    # against the fp64 oracle, full tensors (§8d rule with the committed noise floors)
    # same U as the golden's fp64 run (the fp32 oracle map, upcast)
    u32 = O.uncertainty_map(3, prev, x, 128, 256)
    logits64, final64, _, g64, _ = oracle_run(4, state, x, t, umap=u32, dtype=torch.float64)
    assert (logits.double() - logits64).abs().max().item() <= 1e-3
    sure = logits64.abs() >= 1e-4
    assert torch.equal((torch.sigmoid(logits.double()) > 0.5)[sure], (torch.sigmoid(logits64) > 0.5)[sure])
    print(f"tie band: {int((~sure).sum())} of {sure.numel()} pixels")
    assert abs(final - final64.item()) <= 1e-5 * abs(final64.item())
    bad, ratios, literal, lit_bad, lit_exc = [], [], [], [], []
    for k in param_keys(state):
        g32_max_err, g64_max = (float(v) for v in fx[f"floor/{k}"])
        floor = float(fx[f"floor_pert/{k}"])
        gb = grads[k].double()
        err = (gb - g64[k]).abs().max().item()
        bound = 1e-5 if is_prebn_bias(k) else 3.0 * floor + 1e-6 * g64[k].abs().max().item()
        ratios.append((err / bound, k))
        if err > bound:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
        if is_prebn_bias(k):
            continue  # (true gradient 0: absolute 1e-5 in the survey's rule too)
        # SURVEY §8d's literal rule: max|g - g64| <= 2 max|g32 - g64| + 1e-6 max|g64|, with the
        # reference's own UNPERTURBED fp32 error g32_max_err
        lbound = 2.0 * g32_max_err + 1e-6 * g64_max
        literal.append((err / lbound, k))
        if err > lbound:
            # the reference itself: its fp32 runs with ulp-level weight perturbations err by
            # floor_pert; where that already breaks the literal bound, so may any other
            # equally valid fp32 evaluation order
            (lit_exc if floor > lbound else lit_bad).append(
                f"{k}: {err:.3e} > {lbound:.3e} (reference perturbed-run error {floor:.3e} = "
                f"{floor / lbound:.2f}x the literal bound)")
    ratios.sort(reverse=True)
    literal.sort(reverse=True)
    print("bs16 gradient headroom err/bound: worst", [(round(r, 3), k) for r, k in ratios[:5]],
          "median", round(float(np.median([r for r, _ in ratios])), 4))
    npass = sum(r <= 1.0 for r, _ in literal)
    print(f"SURVEY §8d literal rule (2x unperturbed floor): {npass} of {len(literal)} tensors pass; "
          f"median err/bound {float(np.median([r for r, _ in literal])):.4f}")
    for line in lit_exc:
        print("  literal-rule exception (reference fails it against itself):", line)
    for line in lit_bad:
        print("  LITERAL-RULE FAILURE:", line)
    assert not bad, "gradient parity failures:\n" + "\n".join(bad[:20])
    assert sorted(l.split(":")[0] for l in lit_exc) == sorted(LITERAL_RULE_EXCEPTIONS), \
        ("the literal-rule exceptions changed", [l.split(":")[0] for l in lit_exc])
    assert not lit_bad, "literal §8d rule failures where the reference itself passes:\n" + "\n".join(lit_bad)
    # post-RMSprop parameters: exactly torch's RMSprop rule on the HIP gradients, and the
    # reference's post-step checksums up to the first step's sign flips (RMSprop's first
    # update is ~10 lr * sign(g) whatever |g|, so a noise-level gradient element whose
    # sign differs moves by 2e-3: norm tolerance 1e-4 relative)
    keys = param_keys(state)
    P = {k: state[k].clone() for k in keys}
    O.rmsprop_step(P, {k: grads[k] for k in keys}, {k: torch.zeros_like(P[k]) for k in keys}, 1e-4)
    for k in keys:
        p = sd[k].detach().cpu()
        assert (p - P[k]).abs().max().item() <= 1e-6 * max(1.0, P[k].abs().max().item()), k
        if is_prebn_bias(k):
            continue  # gradient is pure rounding noise (true value 0): every sign is arbitrary
        want = fx[f"post/{k}"]
        assert abs(p.double().norm().item() - want[0]) <= 1e-4 * want[0] + 1e-6, k


def test_config3_bf16_bs16_step(dev):
    """bf16 arithmetic (config 3) at bs16 x 256^2 vs the oracle in the same arithmetic
    (oracle.ref_cpu CONV_MATH = "bf16": bf16 conv operands, fp32 accumulation, conv outputs
    of images >= 32 wide stored in bf16 -- for the U-map stage too), tensor by tensor:
    every gradient within 3x the bf16 oracle's own spread under ulp-level weight
    perturbations (golden G4c, the §8d floor method in bf16) + 1e-6 of its scale; logits
    and loss within 3x their spreads; headroom reported per tensor."""
    from oracle.make_goldens import bf16_oracle_step
    from ugpg import ops
    state, prev, x, t = _inputs()
    fc = np.load("tests/golden/g4c_bf16_floor.npz")
    logits16, final16, u16, g16 = bf16_oracle_step(state, prev, x, t)
    assert abs(final16.item() - fc["loss"][0]) <= 1e-6 * abs(fc["loss"][0]), "oracle drifted"
    fx = np.load("tests/golden/g4b_pgunet4_bs16.npz")
    old = ops.conv_math()
    ops.set_conv_math("bf16")
    try:
        m, logits, ud, final, base, grads = _hip_step(dev, state, prev, x, t)
    finally:
        ops.set_conv_math(old)
    # the U map (Stage-3 forward in bf16)
    assert abs(ud.mean().item() - u16.mean().item()) <= 1e-5
    lerr = (logits - logits16).abs().max().item()
    lbound = 3.0 * fc["floor_logits"][0] + 1e-6 * logits16.abs().max().item()
    assert lerr <= lbound, (lerr, lbound)
    ferr = abs(final - final16.item())
    assert ferr <= 3.0 * fc["floor_loss"][0] + 1e-6 * abs(final16.item()), (ferr, fc["floor_loss"])
    bad, ratios = [], []
    for k in param_keys(state):
        floor, scale = fc[f"floor16/{k}"]
        err = (grads[k].double() - g16[k].double()).abs().max().item()
        bound = 3.0 * floor + 1e-6 * scale
        if is_prebn_bias(k):
            # true value 0 (train-mode BN removes it): pure rounding noise, allowed the fp32
            # test's absolute 1e-5 or the bf16 oracle's own spread, whichever is larger
            # (the image layer's bf16-stored output: spread 2.5e-5, oracle value 2.1e-5)
            bound = max(1e-5, bound)
        ratios.append((err / bound, k))
        if err > bound:
            bad.append(f"{k}: {err:.3e} > {bound:.3e}")
    ratios.sort(reverse=True)
    d = O.dice(O.predictions(logits), t.squeeze(1)).item()
    print(f"bf16 bs16: logits err {lerr:.2e} (bound {lbound:.2e}), loss {final:.6f} vs "
          f"{final16.item():.6f}; gradient headroom err/bound worst "
          f"{[(round(r, 3), k) for r, k in ratios[:5]]}, median "
          f"{float(np.median([r for r, _ in ratios])):.4f}; dice {d:.4f} vs fp32 "
          f"{fx['dice_acc'][0]:.4f}")
    assert not bad, "bf16 gradient parity failures:\n" + "\n".join(bad[:20])
    # the bf16 step against the reference's fp32 one (G4b): the arithmetic's own distance
    assert abs(final - fx["loss"][0]) <= 1e-2 * abs(fx["loss"][0])
    assert abs(d - fx["dice_acc"][0]) <= 1e-2
