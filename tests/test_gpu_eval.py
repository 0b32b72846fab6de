"""Inference / evaluation path (MoNuSegImprove/test_monuseg.py:164-297) on the HIP
kernels vs the CPU oracle restatement (oracle/ref_cpu.py: predict_mask,
calculate_metrics, evaluate_logits).  Parity of the reference module itself is
unpinned (it imports cv2 at top level); its torch calls are the ATen CPU ops."""
import numpy as np
import pytest
import torch

from oracle import detgen as G
from oracle import ref_cpu as O

pytestmark = pytest.mark.gpu

METRICS = ("iou", "dice", "accuracy", "precision", "recall", "specificity")


def _logits(seed, shape, scale=3.0):
    x = G.randn(seed, shape, "x") * scale
    # keep every logit out of the sigmoid(x) > 0.5 tie band (|x| < ~3e-8 rounds to 0.5)
    return torch.where(x.abs() < 1e-4, torch.full_like(x, 1e-3), x)


@pytest.mark.parametrize("B,H,W", [(4, 64, 64), (3, 256, 256), (2, 37, 53)])
def test_seg_eval_matches_calculate_metrics(dev, B, H, W):
    from ugpg import ops
    x = _logits(5, (B, 1, H, W))
    gt = G.bernoulli(6, (B, 1, H, W), 0.3, "t")
    gt[0].zero_()                       # empty ground truth (precision/recall eps paths)
    x[-1] = -x[-1].abs()                # empty prediction in the last sample
    got = ops.seg_eval(x.to(dev), gt.to(dev)).cpu()
    want = O.evaluate_logits(x, gt)
    for b in range(B):
        for i, k in enumerate(METRICS):
            assert np.float32(got[b, i].item()) == want[b][k], (b, k, got[b, i].item(), want[b][k])
        assert abs(got[b, 6].item() - want[b]["confidence"]) <= 1e-6, (b, "confidence")


@pytest.mark.parametrize("H,Ho", [(256, 1000), (256, 200), (64, 128), (32, 32), (50, 77)])
def test_predict_mask_nearest(dev, H, Ho):
    from ugpg import ops
    x = _logits(7, (2, 1, H, H + 3))
    want, _ = O.predict_mask(x, (Ho, Ho + 5))
    got = ops.predict_mask(x.to(dev), (Ho, Ho + 5)).cpu()
    assert torch.equal(got, want)


def test_tester_end_to_end(dev, tmp_path):
    import ugpg
    from tests._parity import det_state
    state = det_state(1, 3, 1)
    torch.save({"model_state_dict": state, "stage": 1, "epoch": 3}, tmp_path / "ckpt.pth")
    tester = ugpg.MoNuSegTester(str(tmp_path / "ckpt.pth"), device=dev)
    assert tester.stage == 1 and not tester.model.training
    x = G.randn(8, (4, 3, 32, 32), "x")
    gt = G.bernoulli(9, (4, 1, 32, 32), 0.4, "t")
    P = {k: v.clone() for k, v in state.items()}
    ref = O.pgunet_forward(1, P, x, training=False)
    # metrics of the oracle's eval-mode logits; a logit inside +-1e-4 may flip a pixel
    want = O.evaluate_logits(ref, gt)
    band = int((ref.abs() < 1e-4).sum())
    avg, std = tester.evaluate_batches([(x[:2], gt[:2]), (x[2:], gt[2:])])
    for k in METRICS:
        vals = np.asarray([w[k] for w in want], dtype=np.float32)
        assert abs(avg[k] - float(np.mean(vals))) <= 1e-6 + band * 2.0 / 1024, k
        assert abs(std[k] - float(np.std(vals))) <= 1e-5 + band * 2.0 / 1024, k
    masks, conf = tester.predict(x, out_size=(50, 40))
    want_m, probs = O.predict_mask(ref, (50, 40))
    assert masks.shape == (4, 1, 50, 40)
    assert int((masks.cpu() != want_m).sum()) <= band * 4
    assert torch.allclose(conf.cpu(), probs.mean(dim=(1, 2, 3)), atol=1e-5)


def test_predict_image_matches_reference_evaluator(dev):
    """MoNuSegEvaluator.predict_image run for real by the golden generator (G10): the
    same resized image tensor through ugpg's tester gives the reference's mask (nearest
    resize back to 45x61) and confidence."""
    import ugpg
    from tests._parity import det_state
    fx = np.load("tests/golden/g10_monuseg_eval.npz")
    state = det_state(1, 3, 1, seed=140)
    model = ugpg.PGUNet1(3, 1)
    model.load_state_dict(state)
    tester = ugpg.MoNuSegTester(model=model, device=dev)
    x = torch.from_numpy(fx["predict_input"])[None]
    masks, conf = tester.predict(x, out_size=(45, 61))
    ref_logits = torch.from_numpy(fx["predict_logits"])
    band = (ref_logits.abs() < 1e-4)
    want = torch.from_numpy(fx["predict_mask"])
    got = masks.cpu().squeeze()
    # pixels whose source logit sits in the +-1e-4 tie band may flip
    from oracle import ref_cpu as O
    src_band, _ = O.predict_mask(band.float() * 10.0, (45, 61))
    sure = src_band.squeeze() == 0
    assert torch.equal(got[sure], want[sure])
    assert abs(conf.item() - float(fx["predict_conf"])) <= 1e-6
