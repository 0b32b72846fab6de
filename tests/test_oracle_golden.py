"""Pin the CPU oracle (oracle/ref_cpu.py) to the reference's own outputs.

The fixtures in tests/golden were produced by oracle/make_goldens.py, which ran
the reference (/root/reference) and the oracle side by side and asserted
torch.equal.  Re-running the oracle here must reproduce them, so the oracle the
GPU tests compare against is the reference's behaviour."""
import json

import numpy as np
import pytest
import torch

from oracle import detgen as G
from oracle import ref_cpu as O
from tests._parity import det_state, is_prebn_bias, oracle_run, param_keys

GOLD = "tests/golden/"


def stats(name, t):
    f = t.detach().double().flatten()
    idx = np.floor(G.uniform(99, 4, name) * f.numel()).astype(np.int64)
    return np.concatenate([[f.pow(2).sum().sqrt().item(), f.sum().item(), f.abs().max().item()],
                           f[idx].numpy()])


def near(a, b, rtol=1e-5, atol=1e-7):
    return np.allclose(np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64),
                       rtol=rtol, atol=atol)


@pytest.mark.parametrize("nc", [1, 2])
def test_g1_pgunet1(nc):
    fx = np.load(GOLD + f"g1_pgunet1_nc{nc}.npz")
    state = det_state(1, 3, nc)
    x = G.randn(1, (4, 3, 32, 32), "x")
    t = G.bernoulli(2, (4, nc, 32, 32), 0.5, "t")
    logits, final, _, g32, P = oracle_run(1, state, x, t)
    assert near(logits.numpy(), fx["logits"], 1e-5, 1e-6)
    assert near(final.numpy(), fx["loss"])
    for k in param_keys(state):
        assert near(stats(k, g32[k]), fx[f"grad32/{k}"], 1e-4, 1e-5 if is_prebn_bias(k) else 1e-9), k
    for k, v in P.items():
        if k.endswith(("running_mean", "running_var")):
            assert near(v.numpy(), fx[f"buf/{k}"]), k
        elif k.endswith("num_batches_tracked"):
            assert int(v) == int(fx[f"buf/{k}"])
    with torch.no_grad():
        ev = O.pgunet_forward(1, P, x, training=False)
    assert near(ev.numpy(), fx["logits_eval"], 1e-5, 1e-6)


def test_g2_uncertainty_maps():
    fx = np.load(GOLD + "g2_umap.npz")
    for prev_stage, B, cur_res in ((1, 2, 64), (3, 2, 256)):
        state = det_state(prev_stage, 3, 1, seed=10 + prev_stage)
        x = G.randn(20 + prev_stage, (B, 3, cur_res, cur_res), "x")
        u = O.uncertainty_map(prev_stage, state, x, O.STAGE_RES[prev_stage], cur_res)
        assert near(u.numpy(), fx[f"s{prev_stage}_u"], 1e-5, 1e-6)
        assert near([u.mean().item(), u.std().item()], fx[f"s{prev_stage}_stats"])


def test_g3_weighted_loss():
    rows = np.load(GOLD + "g3_loss.npz")["rows"]
    out = G.randn(30, (2, 1, 64, 64), "logits")
    t = G.bernoulli(31, (2, 1, 64, 64), 0.3, "t")
    u = torch.from_numpy(G.uniform(32, 2 * 64 * 64, "u").reshape(2, 1, 64, 64)).float()
    for pw, alpha, fin, base in rows:
        f, b = O.weighted_loss(O.bce_pixel(out, t, None if pw == 0 else pw),
                               None if alpha < 0 else u, alpha)
        assert near(f.item(), fin) and near(b, base)


def _g3b_inputs():
    out = G.randn(30, (2, 1, 64, 64), "logits")
    t = G.bernoulli(31, (2, 1, 64, 64), 0.3, "t")
    u = torch.from_numpy(G.uniform(32, 2 * 64 * 64, "u").reshape(2, 1, 64, 64)).float()
    out2 = G.randn(33, (2, 2, 32, 32), "logits2")
    t2 = G.bernoulli(34, (2, 2, 32, 32), 0.3, "t2")
    u2 = torch.from_numpy(G.uniform(35, 2 * 32 * 32, "u2").reshape(2, 1, 32, 32)).float()
    return out, t, u, out2, t2, u2


def test_g3b_weighted_loss_reductions():
    """The reference's weighting for reduction='mean'/'sum' criteria (scalar pixel loss
    broadcast against 1+aU) and 2-channel criteria with per-channel pos_weight/weight."""
    fx = np.load(GOLD + "g3b_loss_reduction.npz")
    out, t, u, out2, t2, u2 = _g3b_inputs()
    n = 0
    for red, pw, use_u, a in O.LOSS_CASES:
        f, b = O.weighted_loss(O.loss_case_criterion(red, pw)(out, t), u if use_u else None, a)
        assert near([f.item(), b], fx[O.loss_case_name(red, pw, use_u, a)]), (red, pw, use_u, a)
        n += 1
    for red, kind in O.LOSS_CASES_C2:
        for use_u in (False, True):
            f, b = O.weighted_loss(O.loss_case_criterion_c2(red, kind)(out2, t2),
                                   u2 if use_u else None, 1.5)
            assert near([f.item(), b], fx[f"c2,red={red},{kind},u={int(use_u)}"])
            n += 1
    assert n == len(fx.files)


def test_g4_logits256_train_mode():
    """The reference's PGUNet4 train-mode logits at 256^2 (bs1) -- the only full-size
    network pin besides the U map."""
    fx = np.load(GOLD + "g4_pgunet4.npz")
    state = det_state(4, 3, 1)
    x256 = G.randn(41, (1, 3, 256, 256), "x256")
    with torch.no_grad():
        o = O.pgunet_forward(4, {k: v.clone() for k, v in state.items()}, x256, training=True)
    assert near(o.numpy(), fx["logits256"], 1e-5, 1e-5)


def test_g4_pgunet4_small():
    fx = np.load(GOLD + "g4_pgunet4.npz")
    state = det_state(4, 3, 1)
    prev = det_state(3, 3, 1, seed=13)
    x = G.randn(1, (2, 3, 64, 64), "x")
    t = G.bernoulli(2, (2, 1, 64, 64), 0.5, "t")
    u = O.uncertainty_map(3, prev, x, 32, 64)
    assert near(u.numpy(), fx["umap"], 1e-5, 1e-6)
    logits, final, base, g32, _ = oracle_run(4, state, x, t, 5.0, u, 1.0)
    assert near(logits.numpy(), fx["logits"], 1e-5, 1e-5)
    assert near([final.item(), base], fx["loss"])
    for k in param_keys(state):
        assert near(stats(k, g32[k]), fx[f"grad32/{k}"], 1e-3, 1e-5 if is_prebn_bias(k) else 1e-8), k


def test_g5_transfer_weights():
    gold = json.load(open(GOLD + "g5_transfer.json"))
    states = {s: det_state(s, 3, 1, seed=50 + s) for s in range(1, 5)}
    for s in (2, 3, 4):
        new, copied = O.transfer_weights(states[s - 1], states[s])
        g = gold[f"{s - 1}->{s}"]
        assert copied == g["copied"]
        for k in copied:
            assert near(float(new[k].double().sum()), g["checksums"][k], 1e-9, 1e-9), k
    assert [len(gold[k]["copied"]) for k in ("1->2", "2->3", "3->4")] == [42, 74, 104]


def test_g6_train_step_tuple():
    gold = json.load(open(GOLD + "g6_train_epoch.json"))
    for stage in (1, 2):
        states = {s: det_state(s, 3, 1, seed=60 + s) for s in (1, 2)}
        res = O.STAGE_RES[stage]
        x = G.randn(61, (4, 3, res, res), "x")
        t = G.bernoulli(62, (4, 1, res, res), 0.5, "t")
        P = {k: v.clone() for k, v in states[stage].items()}
        Pp = {k: v.clone() for k, v in states[stage - 1].items()} if stage > 1 else None
        sq = {k: torch.zeros_like(v) for k, v in P.items() if v.is_floating_point() and not O._is_buffer(k)}
        r = O.ug_train_step(stage, P, Pp, x, t, sq, {1: 3e-4, 2: 1e-4}[stage])
        mine = [r["final_loss"], r["base_loss"], r["dice"], r["acc"], r["unc_mean"], r["unc_std"]]
        assert near(mine, gold[f"stage{stage}"]), (mine, gold[f"stage{stage}"])


def test_g7_herlev():
    fx = np.load(GOLD + "g7_herlev.npz")
    K = 7
    spec = O.state_spec(4, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K)
    state = G.make_state(spec, 70)
    x = G.randn(71, (4, 3, 64, 64), "x")
    le = O.herlev_forward(4, {k: v.clone() for k, v in state.items()}, x, training=False)
    assert near(le.numpy(), fx["logits_eval"], 1e-5, 1e-6)
    y = torch.from_numpy(fx["y"])
    prev = torch.from_numpy(fx["prev_logits"])
    P = {k: v.clone() for k, v in state.items()}
    keys = param_keys(P)
    for k in keys:
        P[k].requires_grad_(True)
    out = O.herlev_forward(4, P, x, training=True)
    f, b, w = O.herlev_ug_loss(out, y, prev, 1.0, K, torch.from_numpy(fx["class_weights"]))
    f.backward()
    assert near([f.item(), b.item()], fx["loss"])
    assert near(w.detach().numpy(), fx["weights"])
    for k in keys:
        if P[k].grad is not None:
            assert near(stats(k, P[k].grad), fx[f"grad32/{k}"], 1e-3, 1e-5 if is_prebn_bias(k) else 1e-8), k


def test_g7b_herlev_trainer_step():
    """The oracle's Herlev step equals the reference HerlevTrainer's own forward pass
    (train_herlev.py:216-296, stage 4 at 224^2, class weights, dropout off)."""
    fx = np.load(GOLD + "g7b_herlev_trainer_step.npz")
    K, cw = 7, torch.from_numpy(fx["class_weights"])
    s4 = G.make_state(O.state_spec(4, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K), 75)
    x = G.randn(77, (4, 3, 224, 224), "x")
    y = G.randint(78, (4,), K, "y")
    assert torch.equal(y, torch.from_numpy(fx["y"]))
    P = {k: v.clone() for k, v in s4.items()}
    keys = param_keys(P)
    for k in keys:
        P[k].requires_grad_(True)
    out = O.herlev_forward(4, P, x, training=True)
    f, b, w = O.herlev_ug_loss(out, y, torch.from_numpy(fx["prev_logits"]), 1.0, K, cw)
    f.backward()
    assert near(out.detach().numpy(), fx["logits"], 1e-5, 1e-6)
    assert near([f.item(), b.item(), w.mean().item(), w.std().item()], fx["loss"])
    for k in keys:
        if P[k].grad is not None:
            assert near(stats(k, P[k].grad), fx[f"grad32/{k}"], 1e-3, 1e-5 if is_prebn_bias(k) else 1e-8), k


def test_g7c_herlev_constructor_rng_parity():
    """ugpg.HerlevClassificationModel draws the reference's probe image at the same point
    of construction: same RNG position afterwards, same initial weights (train_herlev.py:
    48-77).  The probe's BatchNorm update itself runs on the GPU (test_gpu_herlev.py)."""
    from ugpg.herlev import HerlevClassificationModel
    fx = np.load(GOLD + "g7c_herlev_ctor.npz")
    torch.manual_seed(5)
    m = HerlevClassificationModel(stage=4, num_classes=7)
    assert np.array_equal(torch.rand(4).numpy(), fx["rng_after"])
    for k, v in m.state_dict().items():
        if f"sum/{k}" in fx.files:
            # identical weights; the float64 sum's last bits depend on the thread count
            assert near(v.double().sum().item(), float(fx[f"sum/{k}"]), 1e-12, 1e-12), k


def test_g8_dp_shard_semantics_oracle():
    """Mean of per-shard local-BN gradients (the DP step) from the oracle == the
    reference's (G8)."""
    from oracle.make_goldens import G8 as c
    fx = np.load(GOLD + "g8_dp_shards.npz")
    state = det_state(c["stage"], 3, 1, seed=c["w_seed"])
    prev = det_state(c["stage"] - 1, 3, 1, seed=c["prev_seed"])
    x = G.randn(c["x_seed"], (c["B"], 3, c["res"], c["res"]), "x")
    t = G.bernoulli(c["t_seed"], (c["B"], 1, c["res"], c["res"]), 0.5, "t")
    per = c["B"] // c["shards"]
    gs = []
    for r in range(c["shards"]):
        xs, ts = x[r * per:(r + 1) * per], t[r * per:(r + 1) * per]
        u = O.uncertainty_map(1, prev, xs, 32, 64)
        _, _, _, g, _ = oracle_run(c["stage"], state, xs, ts, umap=u)
        gs.append(g)
    for k in param_keys(state):
        avg = sum(g[k] for g in gs) / c["shards"]
        assert near(stats(k, avg), fx[f"avg_grad/{k}"], 1e-3, 1e-5 if is_prebn_bias(k) else 1e-8), k


def test_g9_rng_stream_parity():
    """Building ugpg's ProgressiveUNet / trainer / transfer_weights consumes the global RNG
    exactly like the reference (DataLoader shuffles and augmentation seeds stay in step)."""
    import ugpg
    gold = json.load(open(GOLD + "g9_rng.json"))
    torch.manual_seed(0)
    ugpg.ProgressiveUNet(3, 1)
    assert torch.rand(4).tolist() == gold["after_progressive_unet"]
    torch.manual_seed(1)
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device="cpu")
    assert torch.rand(4).tolist() == gold["after_trainer_ctor"]
    tr.transfer_weights(1, 2)
    assert torch.rand(4).tolist() == gold["after_transfer_1_2"]


def test_g10_monuseg_evaluator_metrics():
    """MoNuSegEvaluator.calculate_metrics run for real (cv2 stubbed when generating):
    the oracle restatement and ugpg's host API reproduce it exactly (float32)."""
    from ugpg.evaluation import calculate_metrics
    fx = np.load(GOLD + "g10_monuseg_eval.npz")
    keys = ("iou", "dice", "accuracy", "precision", "recall", "specificity")
    names = [k.split("/", 1)[1] for k in fx.files if k.startswith("metrics/")]
    assert len(names) == 8
    for n in names:
        want = fx[f"metrics/{n}"]
        for impl in (O.calculate_metrics, calculate_metrics):
            got = impl(fx[f"pred/{n}"], fx[f"gt/{n}"])
            assert [np.float32(got[k]) for k in keys] == [np.float32(v) for v in want], (n, impl)
    # predict_image's mask rule on the reference's own logits
    m, probs = O.predict_mask(torch.from_numpy(fx["predict_logits"]), (45, 61))
    assert np.array_equal(m.squeeze().numpy(), fx["predict_mask"])
    assert probs.mean().item() == float(fx["predict_conf"])
