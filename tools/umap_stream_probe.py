"""Run-to-run determinism of the trainer's U map on a second HIP stream (diagnostic).

Variants, each repeated from the same weights and inputs:
  one      -- the one-stream order (the trainer's);
  side     -- the previous stage's U-map forward on a side stream, concurrent with the
              current stage's forward: its persistent state built first on the current
              stream (prepare_eval), side waits for current, data.record_stream(side),
              current waits for side before the loss, U.record_stream(current) (the
              round-3 experiment, removed from the trainer: DESIGN.md §6a);
  noprep   -- the same ordering rules, but the previous stage's persistent state (flat
              parameters, packs, eval BatchNorm coefficients) is first built ON the side
              stream (no prepare_eval on the current stream);
  serial   -- noprep, but the current stream waits for the side stream before the current
              stage's forward (no kernel concurrency, same allocator traffic);
  naive    -- side stream without side.wait_stream(current), record_stream or prepare.
Prints per step the final loss and the U mean / std of the metrics buffer (exact), so a
variant whose U differs between repetitions or from `one` stands out.

    python tools/umap_stream_probe.py [--steps 4] [--reps 2] [--batch 4]
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path[:0] = [str(ROOT), str(ROOT / "ug-pg-unet_amd")]

import torch  # noqa: E402


def patched_forward(mode):
    from ugpg.loss import weighted_loss_tensors

    def fwd(self, data, target, stage, mbuf):
        cur = torch.cuda.current_stream()
        side = self.__dict__.get("_side") or torch.cuda.Stream()
        self._side = side
        if mode == "side":
            prev = self.models[stage - 1]
            prev.eval()
            prev.prepare_eval()
        if mode != "naive":
            side.wait_stream(cur)
        # (noprep / serial / naive: the previous stage's packs etc. are first built on `side`)
        with torch.cuda.stream(side):
            umap = self.uncertainty_loss.generate_uncertainty_map(
                data, self.models[stage - 1], self.stage_configs[stage - 1]["resolution"],
                self.stage_configs[stage]["resolution"])
        if mode != "naive":
            data.record_stream(side)
        if mode == "serial":
            cur.wait_stream(side)
        output = self.current_model(data)
        cur.wait_stream(side)
        if mode != "naive":
            umap.record_stream(cur)
        final, base = weighted_loss_tensors(self.base_criterion, output, target, umap,
                                            self.uncertainty_alpha, out=mbuf[0:2])
        return output, umap, final, base
    return fwd


def run(variant, steps, B, res=256):
    import ugpg
    from oracle import detgen as G
    from tests._parity import det_state
    dev = torch.device("cuda:0")
    tr = ugpg.UncertaintyGuidedProgressiveTrainer(3, 1, device=dev)
    tr.models[3].load_state_dict(det_state(3, 3, 1, seed=13))
    tr.models[4].load_state_dict(det_state(4, 3, 1, seed=0))
    tr.current_stage, tr.current_model = 4, tr.models[4]
    tr.setup_optimizer(4)
    if variant != "one":
        tr._forward_device = patched_forward(variant).__get__(tr)
    x = G.randn(5, (B, 3, res, res), "x").to(dev)
    t = G.bernoulli(6, (B, 1, res, res), 0.5, "t").to(dev)
    rows = []
    for _ in range(steps):
        d, tt = tr._resize_batch(x * 1.0, t, res)
        rows.append(tr.train_step(d, tt, 4))
    torch.cuda.synchronize()
    return [r.tolist() for r in rows]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--variants", default="one,side,noprep,serial,naive")
    a = ap.parse_args()
    ref = None
    for variant in a.variants.split(","):
        for r in range(a.reps):
            rows = run(variant, a.steps, a.batch)
            ref = rows if ref is None else ref
            same = all(x == y for x, y in zip(rows, ref))
            print(f"{variant} rep {r}: " + " | ".join(
                f"loss {v[0]!r} u {v[5]!r}/{v[6]!r}" for v in rows) +
                f"  {'== first run' if same else '!= first run'}", flush=True)


if __name__ == "__main__":
    main()
