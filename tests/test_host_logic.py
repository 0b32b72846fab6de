"""Host-side logic and API surface of ugpg (CPU only, no kernel launches):
checkpoint format, progressive weight transfer, ProgressiveUNet / trainer /
optimizer API, data-parallel sharding helpers."""
import json

import pytest
import torch
import torch.nn as nn

import ugpg
from oracle import detgen as G
from oracle import ref_cpu as O

GOLD = "tests/golden/"


@pytest.fixture(scope="module")
def spec():
    return json.load(open(GOLD + "g0_state_spec.json"))


@pytest.mark.parametrize("stage", [1, 2, 3, 4])
@pytest.mark.parametrize("nc", [1, 2])
def test_state_dict_matches_reference_checkpoint_format(spec, stage, nc):
    m = getattr(ugpg, f"PGUNet{stage}")(3, nc)
    got = [[k, list(v.shape), str(v.dtype)] for k, v in m.state_dict().items()]
    assert got == spec[f"PGUNet{stage}_nc{nc}"]
    assert sum(p.numel() for p in m.parameters()) == spec["param_counts"][f"PGUNet{stage}"] or nc != 1


def test_progressive_unet_format_and_api(spec):
    pu = ugpg.ProgressiveUNet(3, 1)
    got = [[k, list(v.shape), str(v.dtype)] for k, v in pu.state_dict().items()]
    assert got == spec["ProgressiveUNet"]
    assert pu.current_stage == 1 and pu.get_current_resolution() == 32
    pu.set_stage(3)
    assert pu.get_current_resolution() == 128
    with pytest.raises(ValueError):
        pu.set_stage(5)
    assert pu.stages[4] is pu.stage4
    # README spelling (README.md:46-52) is accepted as an alias
    alias = ugpg.ProgressiveUNet(in_channels=3, out_channels=2, stage=1)
    assert alias.num_classes == 2 and alias.current_stage == 1


def test_reference_checkpoint_loads():
    """A state_dict produced by the reference module layout loads strictly."""
    for stage in (1, 4):
        state = G.make_state(O.state_spec(stage, 3, 1), 5)
        m = getattr(ugpg, f"PGUNet{stage}")(3, 1)
        m.load_state_dict(state, strict=True)
        for k, v in m.state_dict().items():
            assert torch.equal(v, state[k])


def test_transfer_state_matches_reference_golden():
    gold = json.load(open(GOLD + "g5_transfer.json"))
    states = {s: G.make_state(O.state_spec(s, 3, 1), 50 + s) for s in range(1, 5)}
    for s in (2, 3, 4):
        new, copied = ugpg.transfer_state(states[s - 1], states[s])
        g = gold[f"{s - 1}->{s}"]
        assert copied == g["copied"]
        for k in copied:
            assert abs(float(new[k].double().sum()) - g["checksums"][k]) <= 1e-9 * max(1, abs(g["checksums"][k]))
        assert list(new.keys()) == list(states[s].keys())


def test_progressive_transfer_weights_prints_and_returns(capsys):
    pu = ugpg.ProgressiveUNet(3, 1)
    new = pu.transfer_weights(pu.stage1.state_dict(), pu.stage2.state_dict(), 2)
    assert "copied 42 keys" in capsys.readouterr().out
    pu.stage2.load_state_dict(new)


def test_trainer_public_surface_on_cpu():
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device="cpu", uncertainty_alpha=0.5)
    assert set(tr.stage_configs) == {1, 2, 3, 4}
    assert [tr.stage_configs[s]["resolution"] for s in (1, 2, 3, 4)] == [32, 64, 128, 256]
    assert [tr.stage_configs[s]["lr"] for s in (1, 2, 3, 4)] == [3e-4, 1e-4, 1e-4, 1e-4]
    assert set(tr.models) == {1, 2, 3, 4} and tr.current_model is tr.models[1]
    assert isinstance(tr.base_criterion, nn.BCEWithLogitsLoss)
    assert tr.base_criterion.pos_weight.item() == 5.0 and tr.base_criterion.reduction == "none"
    assert isinstance(tr.optimizer, ugpg.RMSprop)
    assert tr.optimizer.param_groups[0]["weight_decay"] == 1e-4
    assert set(tr.history) == {"train_loss", "val_loss", "train_dice", "val_dice",
                               "uncertainty_weights_mean", "uncertainty_weights_std",
                               "base_loss", "stage_transitions"}
    for name in ("setup_optimizer", "dice_coefficient", "get_predictions", "calculate_accuracy",
                 "transfer_weights", "uncertainty_guided_forward_pass", "train_epoch",
                 "validate_epoch", "train_progressive", "save_training_plots",
                 "load_stage_weights", "save_uncertainty_analysis"):
        assert callable(getattr(tr, name))
    # host-side metric helpers keep the reference semantics
    pred = torch.tensor([[[1.0, 0.0], [1.0, 1.0]]])
    tgt = torch.tensor([[[1.0, 0.0], [0.0, 1.0]]])
    assert abs(tr.dice_coefficient(pred, tgt).item() - (2 * 2 + 1) / (3 + 2 + 1)) < 1e-7
    assert tr.calculate_accuracy(pred, tgt.long()) == 0.75
    # subclass contract (train_aug_monuseg.py:42-121): replace criterion and epochs
    tr.base_criterion = nn.BCEWithLogitsLoss(pos_weight=torch.tensor([3.2]), reduction="none")
    for s in tr.stage_configs:
        tr.stage_configs[s]["epochs_per_stage"] = 2
    tr.transfer_weights(1, 2)


def test_v1_helper_and_aliases():
    from ugpg import UG_unet, UG_unet_parts, uncertainty_guided_trainer
    h = UG_unet.UncertaintyGuidedProgressiveTrainer(device="cpu")
    assert h.stage_resolutions == {1: 32, 2: 64, 3: 128, 4: 256}
    fn = h.create_uncertainty_weighted_loss_fn(nn.BCEWithLogitsLoss(pos_weight=torch.tensor([2.0])))
    assert fn.reduction == "none" and fn.pos_weight.item() == 2.0
    assert UG_unet_parts.Up is ugpg.Up and uncertainty_guided_trainer.UncertaintyGuidedProgressiveTrainer \
        is ugpg.UncertaintyGuidedProgressiveTrainer


def test_rmsprop_rejects_unsupported_configs():
    p = [nn.Parameter(torch.zeros(3))]
    with pytest.raises(NotImplementedError):
        ugpg.RMSprop(p, lr=1e-3, momentum=0.9)
    with pytest.raises(NotImplementedError):
        ugpg.RMSprop(p, lr=1e-3, centered=True)
    opt = ugpg.RMSprop(p, lr=1e-3, weight_decay=1e-4)
    assert opt.state_dict()["param_groups"][0]["alpha"] == 0.99


def test_models_refuse_cpu_execution():
    m = ugpg.PGUNet1(3, 1)
    with pytest.raises(RuntimeError, match="ROCm"):
        m(torch.zeros(1, 3, 32, 32))


@pytest.mark.parametrize("stage", [1, 2, 3, 4])
def test_herlev_model_checkpoint_format(stage):
    """Key layout of the reference HerlevClassificationModel (train_herlev.py:29-121);
    the oracle spec is pinned by g7 (loaded strictly into the reference model)."""
    from ugpg.herlev import HerlevClassificationModel
    m = HerlevClassificationModel(stage, 7)
    want = [k for k, _, _ in O.state_spec(stage, 3, 1, key_prefix="unet.")]
    want += [k for k, _, _ in O.herlev_head_spec(512, 7)]
    assert list(m.state_dict().keys()) == want
    state = G.make_state(O.state_spec(stage, 3, 1, key_prefix="unet.") + O.herlev_head_spec(512, 7), 3)
    m.load_state_dict(state, strict=True)


def test_shard_helper():
    from ugpg.dist import shard
    x = torch.arange(16).view(16, 1)
    parts = [shard(x, r, 4) for r in range(4)]
    assert torch.equal(torch.cat(parts), x)
    with pytest.raises(ValueError):
        shard(x, 0, 3)


def test_eval_metrics_host_api_matches_oracle():
    """ugpg.evaluation.calculate_metrics keeps test_monuseg.py:264-297's numpy float32
    arithmetic (the oracle restatement) exactly, including the empty-mask eps paths."""
    import numpy as np
    from ugpg.evaluation import calculate_metrics
    rng = np.random.default_rng(0)
    cases = [(rng.random(4096) > 0.5, rng.random(4096) > 0.7),
             (np.zeros(100), rng.random(100) > 0.5), (rng.random(100) > 0.5, np.zeros(100)),
             (np.zeros(64), np.zeros(64)), (np.ones(64), np.ones(64))]
    for pred, gt in cases:
        got = calculate_metrics(pred.astype(np.float32), gt.astype(np.float32))
        want = O.calculate_metrics(pred, gt)
        for k, v in want.items():
            assert got[k] == v and type(got[k]) is type(v), k


def test_tester_checkpoint_formats(tmp_path):
    """MoNuSegTester.load_model (test_monuseg.py:120-162): checkpoint dict with 'stage',
    raw state_dict (stage 4), anything else rejected; weights-only loading."""
    import ugpg
    from tests._parity import det_state
    s2 = det_state(2, 3, 1)
    torch.save({"model_state_dict": s2, "stage": 2, "val_dice": 0.5}, tmp_path / "a.pth")
    t = ugpg.MoNuSegTester(str(tmp_path / "a.pth"), device="cpu")
    assert t.stage == 2 and isinstance(t.model, ugpg.PGUNet2) and not t.model.training
    s4 = det_state(4, 3, 1)
    torch.save(s4, tmp_path / "b.pth")
    t = ugpg.MoNuSegTester(str(tmp_path / "b.pth"), device="cpu")
    assert t.stage == 4 and isinstance(t.model, ugpg.PGUNet4)
    torch.save([1, 2, 3], tmp_path / "c.pth")
    with pytest.raises(RuntimeError, match="Unrecognized checkpoint"):
        ugpg.MoNuSegTester(str(tmp_path / "c.pth"), device="cpu")


def test_herlev_progressive_driver_early_stop_and_scheduler(tmp_path, monkeypatch):
    """train_herlev.py:404-489 control flow with scripted epoch results: the
    scheduler steps on val_loss (factor 0.5 after 5 bad epochs), a checkpoint is
    written on each val_acc improvement, early stop after `early_stopping_patience`
    stale epochs, history JSON with the reference's keys."""
    from ugpg.herlev import HerlevTrainer
    cfg = {"device": "cpu", "epochs_per_stage": 12, "num_classes": 7, "stages": [1, 2],
           "early_stopping_patience": 8}
    tr = HerlevTrainer(cfg)
    script = {1: [(1.0, 10.0)] + [(1.0, 5.0)] * 11,             # (val_loss, val_acc)
              2: [(2.0, 1.0), (1.5, 2.0), (1.0, 3.0)] + [(1.0, 3.0)] * 9}
    calls = {1: 0, 2: 0}

    def train_epoch(loader, stage):
        return (0.5, 0.4, 50.0, 0.0, 0.0)

    def validate_epoch(loader, stage):
        vl, va = script[stage][calls[stage]]
        calls[stage] += 1
        return (vl, vl, va, 1.0, 0.0)

    monkeypatch.setattr(tr, "train_epoch", train_epoch)
    monkeypatch.setattr(tr, "validate_epoch", validate_epoch)
    tr.train_progressive({1: None, 2: None}, {1: None, 2: None}, str(tmp_path))
    assert calls == {1: 9, 2: 11}          # best at epoch 1 (3), then 8 stale epochs
    assert tr.optimizers[1].param_groups[0]["lr"] == pytest.approx(1.5e-4)   # halved once
    assert tr.optimizers[2].param_groups[0]["lr"] == pytest.approx(5e-5)
    ck = torch.load(tmp_path / "herlev_stage2_best.pth", weights_only=True)
    assert ck["epoch"] == 3 and ck["val_acc"] == 3.0 and ck["stage"] == 2
    assert set(ck) == {"model_state_dict", "optimizer_state_dict", "stage", "epoch",
                       "train_loss", "val_loss", "train_acc", "val_acc", "config"}
    h = json.loads((tmp_path / "training_history.json").read_text())
    assert len(h["val_loss"]) == 20 and h["base_loss"][0] == 1.0
    assert [t["stage"] for t in h["stage_transitions"]] == [1, 2]
    assert h["stage_transitions"][0]["best_val_acc"] == 10.0
