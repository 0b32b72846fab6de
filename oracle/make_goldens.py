"""Generate and pin the golden fixtures (RUNS IN THE BUILD CONTAINER ONLY).

Imports the reference from /root/reference (read-only), drives it and the
oracle (`oracle/ref_cpu.py`) with identical deterministic weights and inputs,
asserts they agree (torch.equal on CPU: same ops, same order), and writes small
fixtures to tests/golden/.  Nothing from the reference is copied: only tensors,
key lists and scalars produced by running it.

    python -m oracle.make_goldens

Fixture map:
  g1_pgunet1_nc{1,2}.npz  PGUNet1 bs4 32^2: logits (train/eval), BCE loss, per-param
                          grad stats + fp64 noise floor, BN running stats, post-RMSprop stats
  g2_umap.npz             uncertainty maps S1@32->64 and S3@128->256, bs2
  g3_loss.npz             weighted loss for alpha in {0,.5,1,2,5}
  g4_pgunet4.npz          PGUNet4 bs2 64^2 (+ bs1 256^2 logits), UG loss w/ S3 map, grads
  g5_transfer.json        transfer_weights 1->2, 2->3, 3->4 copied keys + checksums
  g6_train_epoch.json     trainer.train_epoch 6-tuples, stage 1 and stage 2
  g7_herlev.npz           Herlev S4 classifier (eval logits, UG CE loss, grads w/o dropout)
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn as nn

from oracle import detgen as G
from oracle import ref_cpu as O

REF = "/root/reference"
OUT = Path(__file__).resolve().parent.parent / "tests" / "golden"
W_SEED, X_SEED, T_SEED = 0, 1, 2
N_SAMPLES = 4


def _ref():
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import UG_unet as RU  # noqa: E402
    return RU


def det_state(stage, in_ch, nc, seed=W_SEED, key_prefix=""):
    return G.make_state(O.state_spec(stage, in_ch, nc, key_prefix), seed)


def sample_idx(name, n):
    return np.floor(G.uniform(99, N_SAMPLES, name) * n).astype(np.int64)


def tstats(name, t):
    f = t.detach().double().flatten()
    idx = sample_idx(name, f.numel())
    return np.concatenate([[f.pow(2).sum().sqrt().item(), f.sum().item(), f.abs().max().item()],
                           f[idx].numpy()])


def param_keys(state):
    return [k for k, v in state.items() if v.is_floating_point() and not O._is_buffer(k)]


def oracle_grads(stage, state, x, t, pos_weight, umap=None, alpha=1.0, dtype=torch.float32):
    P = {k: v.clone().to(dtype) if v.is_floating_point() else v.clone() for k, v in state.items()}
    keys = param_keys(P)
    for k in keys:
        P[k].requires_grad_(True)
    logits = O.pgunet_forward(stage, P, x.to(dtype), training=True)
    u = None if umap is None else umap.to(dtype)
    final, base = O.weighted_loss(O.bce_pixel(logits, t.to(dtype), pos_weight), u, alpha)
    final.backward()
    return logits.detach(), final.detach(), base, {k: P[k].grad.detach() for k in keys}, P


def save_npz(name, **arrays):
    OUT.mkdir(parents=True, exist_ok=True)
    np.savez_compressed(OUT / name, **{k: np.asarray(v) for k, v in arrays.items()})
    print("wrote", name, f"{(OUT / name).stat().st_size / 1024:.0f} KiB")


def grad_fixture(prefix, keys, g32, g64):
    out = {}
    for k in keys:
        out[f"{prefix}grad32/{k}"] = tstats(k, g32[k])
        out[f"{prefix}grad64/{k}"] = tstats(k, g64[k])
        out[f"{prefix}floor/{k}"] = np.array([(g32[k].double() - g64[k]).abs().max().item(),
                                             g64[k].abs().max().item()])
    return out


# ---------------------------------------------------------------------------

def g1(RU, nc):
    stage, B, res = 1, 4, 32
    state = det_state(stage, 3, nc)
    x = G.randn(X_SEED, (B, 3, res, res), "x")
    t = G.bernoulli(T_SEED, (B, nc, res, res), 0.5, "t")
    ref = RU.PGUNet1(3, nc)
    ref.load_state_dict(state)
    # train-mode forward/backward through the reference
    ref.train()
    out_ref = ref(x)
    crit = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([5.0]), reduction="none")
    loss_ref = torch.mean(crit(out_ref, t))
    loss_ref.backward()
    logits, final, _, g32, P = oracle_grads(stage, state, x, t, 5.0)
    assert torch.equal(logits, out_ref.detach()), "G1: oracle logits != reference"
    assert torch.equal(final, loss_ref.detach()), "G1: oracle loss != reference"
    for k, p in ref.named_parameters():
        assert torch.equal(g32[k], p.grad), f"G1: grad {k} differs"
    for k, v in ref.state_dict().items():
        assert torch.equal(v, P[k].detach()), f"G1: buffer/param {k} differs after fwd"
    _, _, _, g64, _ = oracle_grads(stage, state, x, t, 5.0, dtype=torch.float64)
    # eval-mode logits (running stats as updated by the train forward)
    ref.eval()
    with torch.no_grad():
        eval_ref = ref(x)
        P_eval = {k: v.detach() for k, v in P.items()}
        eval_o = O.pgunet_forward(stage, P_eval, x, training=False)
    assert torch.equal(eval_ref, eval_o)
    # one RMSprop step (lr 3e-4, stage 1) through torch.optim on the reference params
    opt = torch.optim.RMSprop(ref.parameters(), lr=3e-4, weight_decay=1e-4)
    opt.step()
    keys = param_keys(state)
    Pn = {k: P[k].detach().clone() for k in keys}
    sq = {k: torch.zeros_like(Pn[k]) for k in keys}
    O.rmsprop_step(Pn, g32, sq, 3e-4)
    sd = ref.state_dict()
    for k in keys:
        assert torch.equal(Pn[k], sd[k]), f"G1: post-RMSprop {k} differs"
    fx = dict(x_sum=x.sum().numpy(), t_sum=t.sum().numpy(), logits=logits.numpy(),
              logits_eval=eval_ref.numpy(), loss=final.numpy(), loss64=np.array(0.0))
    fx.update(grad_fixture("", keys, g32, g64))
    for k in keys:
        fx[f"post/{k}"] = tstats(k, Pn[k])
    for k, v in sd.items():
        if O._is_buffer(k) and v.is_floating_point():
            fx[f"buf/{k}"] = v.numpy()
        elif k.endswith("num_batches_tracked"):
            fx[f"buf/{k}"] = np.array(int(v))
    save_npz(f"g1_pgunet1_nc{nc}.npz", **fx)


def g2(RU):
    fx = {}
    loss_mod = RU.UncertaintyGuidedLoss(device="cpu")
    for prev_stage, B, cur_res in ((1, 2, 64), (3, 2, 256)):
        prev_res = O.STAGE_RES[prev_stage]
        state = det_state(prev_stage, 3, 1, seed=10 + prev_stage)
        x = G.randn(20 + prev_stage, (B, 3, cur_res, cur_res), "x")
        ref = getattr(RU, f"PGUNet{prev_stage}")(3, 1)
        ref.load_state_dict(state)
        u_ref = loss_mod.generate_uncertainty_map(x, ref, prev_res, cur_res)
        u_o = O.uncertainty_map(prev_stage, state, x, prev_res, cur_res)
        assert torch.equal(u_ref, u_o), f"G2: umap differs (prev stage {prev_stage})"
        fx[f"s{prev_stage}_u"] = u_o.numpy()
        fx[f"s{prev_stage}_stats"] = np.array([u_o.mean().item(), u_o.std().item()])
    save_npz("g2_umap.npz", **fx)


def g3(RU):
    loss_mod = RU.UncertaintyGuidedLoss(device="cpu")
    out = G.randn(30, (2, 1, 64, 64), "logits")
    t = G.bernoulli(31, (2, 1, 64, 64), 0.3, "t")
    u = torch.from_numpy(G.uniform(32, 2 * 64 * 64, "u").reshape(2, 1, 64, 64)).float()
    rows = []
    for pw in (None, 5.0):
        crit = nn.BCEWithLogitsLoss(pos_weight=None if pw is None else torch.tensor([pw]),
                                    reduction="none")
        for alpha in (0.0, 0.5, 1.0, 2.0, 5.0):
            f_ref, b_ref = loss_mod.apply_uncertainty_weighted_loss(crit, out, t, u, alpha)
            f_o, b_o = O.weighted_loss(O.bce_pixel(out, t, pw), u, alpha)
            assert torch.equal(f_ref, f_o) and b_ref == b_o
            rows.append([0.0 if pw is None else pw, alpha, f_o.item(), b_o])
        f_ref, b_ref = loss_mod.apply_uncertainty_weighted_loss(crit, out, t, None, 1.0)
        f_o, b_o = O.weighted_loss(O.bce_pixel(out, t, pw), None)
        assert torch.equal(f_ref, f_o)
        rows.append([0.0 if pw is None else pw, -1.0, f_o.item(), b_o])
    save_npz("g3_loss.npz", rows=np.array(rows))


def g4(RU):
    fx = {}
    state = det_state(4, 3, 1)
    prev = det_state(3, 3, 1, seed=13)
    B, res = 2, 64
    x = G.randn(X_SEED, (B, 3, res, res), "x")
    t = G.bernoulli(T_SEED, (B, 1, res, res), 0.5, "t")
    loss_mod = RU.UncertaintyGuidedLoss(device="cpu")
    ref_prev = RU.PGUNet3(3, 1)
    ref_prev.load_state_dict(prev)
    u_ref = loss_mod.generate_uncertainty_map(x, ref_prev, res // 2, res)
    u = O.uncertainty_map(3, prev, x, res // 2, res)
    assert torch.equal(u, u_ref)
    ref = RU.PGUNet4(3, 1)
    ref.load_state_dict(state)
    out_ref = ref(x)
    crit = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([5.0]), reduction="none")
    f_ref, b_ref = loss_mod.apply_uncertainty_weighted_loss(crit, out_ref, t, u_ref, 1.0)
    f_ref.backward()
    logits, final, base, g32, P = oracle_grads(4, state, x, t, 5.0, u, 1.0)
    assert torch.equal(logits, out_ref.detach()) and torch.equal(final, f_ref.detach())
    assert base == b_ref
    for k, p in ref.named_parameters():
        assert torch.equal(g32[k], p.grad), f"G4: grad {k} differs"
    _, final64, _, g64, _ = oracle_grads(4, state, x, t, 5.0, u, 1.0, dtype=torch.float64)
    keys = param_keys(state)
    fx.update(grad_fixture("", keys, g32, g64))
    fx.update(logits=logits.numpy(), umap=u.numpy(), loss=np.array([final.item(), base]),
              loss64=np.array(final64.item()))
    ref.eval()
    with torch.no_grad():
        fx["logits_eval"] = ref(x).numpy()
        x256 = G.randn(41, (1, 3, 256, 256), "x256")
        ref.train()
        o256 = ref(x256)
        Pn = {k: v.detach().clone() for k, v in state.items()}
        # ref already ran one train forward on `state` buffers -> use fresh copy for oracle
        ref2 = RU.PGUNet4(3, 1)
        ref2.load_state_dict(state)
        o256_ref = ref2(x256)
        o256_o = O.pgunet_forward(4, Pn, x256, training=True)
        assert torch.equal(o256_ref, o256_o)
        fx["logits256"] = o256_o.numpy()
    save_npz("g4_pgunet4.npz", **fx)


def g5(RU):
    import uncertainty_guided_trainer as RT  # noqa: E402
    states = {s: det_state(s, 3, 1, seed=50 + s) for s in range(1, 5)}
    out = {}
    pu = RU.ProgressiveUNet(3, 1)
    for s in (2, 3, 4):
        new_ref = pu.transfer_weights(states[s - 1], states[s], s)
        new_o, copied = O.transfer_weights(states[s - 1], states[s])
        assert list(new_ref.keys()) == list(new_o.keys())
        for k in new_ref:
            assert torch.equal(new_ref[k], new_o[k]), f"G5: {k}"
        out[f"{s - 1}->{s}"] = dict(copied=copied,
                                    checksums={k: float(new_o[k].double().sum()) for k in copied})
    _ = RT
    (OUT / "g5_transfer.json").write_text(json.dumps(out, indent=1))
    print("wrote g5_transfer.json", {k: len(v["copied"]) for k, v in out.items()})


def g6(RU):
    import uncertainty_guided_trainer as RT  # noqa: E402
    from torch.utils.data import DataLoader, TensorDataset
    res_all = {}
    for stage in (1, 2):
        torch.manual_seed(0)
        tr = RT.UncertaintyGuidedProgressiveTrainer(3, 1, device="cpu", uncertainty_alpha=1.0)
        states = {s: det_state(s, 3, 1, seed=60 + s) for s in (1, 2)}
        for s in (1, 2):
            tr.models[s].load_state_dict(states[s])
        tr.current_stage = stage
        tr.current_model = tr.models[stage]
        tr.setup_optimizer(stage)
        res = O.STAGE_RES[stage]
        x = G.randn(61, (4, 3, res, res), "x")
        t = G.bernoulli(62, (4, 1, res, res), 0.5, "t")
        loader = DataLoader(TensorDataset(x, t), batch_size=4)
        tup = tr.train_epoch(loader, stage)
        # oracle
        P = {k: v.clone() for k, v in states[stage].items()}
        Pp = {k: v.clone() for k, v in states[stage - 1].items()} if stage > 1 else None
        sq = {k: torch.zeros_like(v) for k, v in P.items() if v.is_floating_point() and not O._is_buffer(k)}
        r = O.ug_train_step(stage, P, Pp, x, t, sq, O_LR[stage])
        mine = (r["final_loss"], r["base_loss"], r["dice"], r["acc"], r["unc_mean"], r["unc_std"])
        assert tuple(float(a) for a in tup) == tuple(float(a) for a in mine), (tup, mine)
        for k, v in tr.models[stage].state_dict().items():
            assert torch.equal(v, P[k].detach()), f"G6: {k} after step"
        res_all[f"stage{stage}"] = [float(a) for a in tup]
    (OUT / "g6_train_epoch.json").write_text(json.dumps(res_all, indent=1))
    print("wrote g6_train_epoch.json", res_all)


O_LR = {1: 3e-4, 2: 1e-4, 3: 1e-4, 4: 1e-4}


def g7(RU):
    # Herlev imports torchvision only for its dataset module: stub it in-process.
    import types
    for mod in ("torchvision", "torchvision.transforms", "herlev_dataset"):
        if mod not in sys.modules:
            m = types.ModuleType(mod)
            m.HerlevDataset = object
            m.transforms = m
            sys.modules[mod] = m
    sys.path.insert(0, os.path.join(REF, "Herlev"))
    import train_herlev as H  # noqa: E402
    K, B, res = 7, 4, 64
    ref = H.HerlevClassificationModel(stage=4, num_classes=K)
    spec = O.state_spec(4, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K)
    state = G.make_state(spec, 70)
    ref.load_state_dict(state)
    x = G.randn(71, (B, 3, res, res), "x")
    y = G.randint(72, (B,), K, "y")
    ref.eval()
    with torch.no_grad():
        le_ref = ref(x)
    le = O.herlev_forward(4, {k: v.clone() for k, v in state.items()}, x, training=False)
    assert torch.equal(le, le_ref)
    # train mode, dropout disabled on both sides -> deterministic; BN in train mode
    ref.train()
    for m in ref.modules():
        if isinstance(m, nn.Dropout):
            m.p = 0.0
    ref_prev = H.HerlevClassificationModel(stage=3, num_classes=K)
    state_prev = G.make_state(O.state_spec(3, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, K), 73)
    ref_prev.load_state_dict(state_prev)
    ref_prev.eval()
    with torch.no_grad():
        prev_logits = ref_prev(torch.nn.functional.interpolate(x, size=(res // 2, res // 2),
                                                               mode="bilinear", align_corners=True))
    out = ref(x)
    cw = torch.linspace(0.5, 2.0, K)
    f_ref, b_ref, w_ref = O.herlev_ug_loss(out, y, prev_logits, 1.0, K, cw)
    f_ref.backward()
    P = {k: v.clone() for k, v in state.items()}
    keys = [k for k in param_keys(P)]
    for k in keys:
        P[k].requires_grad_(True)
    out_o = O.herlev_forward(4, P, x, training=True)
    f_o, b_o, w_o = O.herlev_ug_loss(out_o, y, prev_logits, 1.0, K, cw)
    f_o.backward()
    assert torch.equal(out_o, out) and torch.equal(f_o, f_ref)
    fx = dict(logits_eval=le.numpy(), logits_train=out_o.detach().numpy(),
              prev_logits=prev_logits.numpy(), loss=np.array([f_o.item(), b_o.item()]),
              weights=w_o.numpy(), y=y.numpy(), class_weights=cw.numpy())
    for k, p in ref.named_parameters():
        if p.grad is None:  # decoder/head of the wrapped PGUNet4 is unused by the classifier
            assert P[k].grad is None, f"G7 grad {k}"
            continue
        assert torch.equal(P[k].grad, p.grad), f"G7 grad {k}"
        fx[f"grad32/{k}"] = tstats(k, p.grad)
    save_npz("g7_herlev.npz", **fx)


def g0(RU):
    """state_dict keys/shapes/dtypes of every reference model (checkpoint format)."""
    out = {}
    for stage in (1, 2, 3, 4):
        for nc in (1, 2):
            m = getattr(RU, f"PGUNet{stage}")(3, nc)
            out[f"PGUNet{stage}_nc{nc}"] = [[k, list(v.shape), str(v.dtype)]
                                           for k, v in m.state_dict().items()]
    pu = RU.ProgressiveUNet(3, 1)
    out["ProgressiveUNet"] = [[k, list(v.shape), str(v.dtype)] for k, v in pu.state_dict().items()]
    out["param_counts"] = {f"PGUNet{s}": sum(p.numel() for p in getattr(RU, f"PGUNet{s}")(3, 1).parameters())
                           for s in (1, 2, 3, 4)}
    (OUT / "g0_state_spec.json").write_text(json.dumps(out))
    print("wrote g0_state_spec.json", out["param_counts"])


def main():
    torch.set_num_threads(8)
    RU = _ref()
    g0(RU)
    g1(RU, 1)
    g1(RU, 2)
    g2(RU)
    g3(RU)
    g4(RU)
    g5(RU)
    g6(RU)
    g7(RU)


if __name__ == "__main__":
    main()
